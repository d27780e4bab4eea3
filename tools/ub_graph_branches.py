"""Do parallel branches of a captured hipGraph run concurrently on MI355X?"""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops

dev = "cuda"
a = torch.randn(512, 512, device=dev, dtype=torch.bfloat16)
bs = [torch.randn(512, 512, device=dev, dtype=torch.bfloat16) for _ in range(2)]
n = 200


def chain(b):
    x = a
    for _ in range(n):
        x = ops.linear_fwd(x, b)
    return x


def timed(fn, reps=5):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


chain(bs[0]); torch.cuda.synchronize()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
# one chain in a graph
g1 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g1):
    chain(bs[0])
# two chains on one stream (serial)
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    chain(bs[0]); chain(bs[1])
# two chains on two branches
g3 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g3):
    main = torch.cuda.current_stream()
    s1.wait_stream(main); s2.wait_stream(main)
    with torch.cuda.stream(s1):
        chain(bs[0])
    with torch.cuda.stream(s2):
        chain(bs[1])
    main.wait_stream(s1); main.wait_stream(s2)
print(f"1 chain {timed(g1.replay):.2f} ms; 2 chains serial {timed(g2.replay):.2f} ms; "
      f"2 chains as graph branches {timed(g3.replay):.2f} ms")


# eager two streams
def eager2():
    main = torch.cuda.current_stream()
    s1.wait_stream(main); s2.wait_stream(main)
    with torch.cuda.stream(s1):
        chain(bs[0])
    with torch.cuda.stream(s2):
        chain(bs[1])
    main.wait_stream(s1); main.wait_stream(s2)


print(f"eager: 1 chain {timed(lambda: chain(bs[0])):.2f} ms; 2 streams {timed(eager2):.2f} ms")
