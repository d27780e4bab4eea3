"""Diffusion algorithms: sqrt schedule, DDIM / cold samplers, img2img."""
from .schedule import (alpha_bar_train, cold_steps, ddim_coefficients, ddim_table, ddim_timesteps,
                       img2img_alpha)
from .samplers import ColdSampler, DDIMSampler, img2img

__all__ = ["alpha_bar_train", "cold_steps", "ddim_coefficients", "ddim_table", "ddim_timesteps",
           "img2img_alpha", "ColdSampler", "DDIMSampler", "img2img"]
