"""A/B of a module-level constant on one box: bench.py's training step with
<module>.<NAME> set to each value in turn, interleaved REPS times.
usage: python tools/ab_module_constant.py <module> <NAME> <v1,v2> [reps] -- <bench.py args>"""
import contextlib
import importlib
import io
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

sep = sys.argv.index("--")
mod_name, name, vals = sys.argv[1], sys.argv[2], [int(v) for v in sys.argv[3].split(",")]
reps = int(sys.argv[4]) if sep > 4 else 2
args = sys.argv[sep + 1:]
mod = importlib.import_module(mod_name)
orig = getattr(mod, name)
for _ in range(reps):
    for v in vals:
        setattr(mod, name, v)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            bench.main(args)
        line = [l for l in buf.getvalue().splitlines() if l.startswith("{")][-1]
        print(f"{name}={v}: {json.loads(line)['ms_per_step']} ms/step", flush=True)
setattr(mod, name, orig)
