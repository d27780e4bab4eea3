"""Benchmark helpers (eager PyTorch comparators for the headline numbers)."""
