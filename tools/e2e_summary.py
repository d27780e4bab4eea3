"""Summarise a trainer log's `# perf:` lines (ddim_cold_amd/train/trainer.py) as markdown:
steady-state step rate (median of the device-timed log windows), every epoch's
end-to-end rate with its evaluation / checkpoint hand-off / background write times,
the window that contains each epoch boundary relative to the steady window, and the
whole run's end-to-end rate as a fraction of the steady rate.
usage: python tools/e2e_summary.py train.log [title]"""
import re
import statistics
import sys

WIN = re.compile(r"# perf: ([\d.]+) img/s\s+([\d.]+) ms/step \(device")
STEPS = re.compile(r"steps:\s+(\d+) loss: ([\d.]+) time_cost: ([\d.]+)")
EPOCH = re.compile(r"# perf: epoch (\d+) end to end ([\d.]+) img/s \(([\d.]+) s: evaluate ([\d.]+) ms, "
                   r"checkpoint hand-off ([\d.]+) ms, previous write ([\d.]+) ms")
PARTS = re.compile(r"host copy wait ([\d.]+), layout ([\d.]+), files ([\d.]+)")
RUN = re.compile(r"# perf: run end to end ([\d.]+) img/s over (\d+) steps \(([\d.]+) s")
EPOCH_LINE = re.compile(r"^epoch:\s+(\d+)")


def main(path, title=None):
    lines = open(path).read().splitlines()
    windows = []  # (img/s, ms/step, wall s of the window, contains an epoch boundary)
    epochs, run = [], None
    boundary = False
    last_wall = None
    for ln in lines:
        if EPOCH_LINE.match(ln):
            boundary = True
        m = STEPS.search(ln)
        if m:
            last_wall = float(m.group(3))
            continue
        m = WIN.search(ln)
        if m:
            windows.append((float(m.group(1)), float(m.group(2)), last_wall, boundary))
            boundary = False
            continue
        m = EPOCH.search(ln)
        if m:
            p = PARTS.search(ln)
            epochs.append(tuple(float(v) for v in m.groups()) + (p.group(0) if p else "",))
            continue
        m = RUN.search(ln)
        if m:
            run = (float(m.group(1)), int(m.group(2)), float(m.group(3)))
    steady = [w for w in windows[1:] if not w[3]]  # the first window holds the graph capture
    if not steady:
        print("no steady-state windows found")
        return 1
    st_rate = statistics.median(w[0] for w in steady)
    st_ms = statistics.median(w[1] for w in steady)
    st_wall = statistics.median(w[2] for w in steady if w[2] is not None)
    out = [f"# {title or path}", "",
           f"Steady state (median of {len(steady)} device-timed log windows without an epoch boundary): "
           f"**{st_rate:,.1f} img/s**, {st_ms:.3f} ms/step, {st_wall:.2f} s host wall per window.", ""]
    bw = [w for w in windows[1:] if w[3]]
    if bw:
        r = [w[2] / st_wall for w in bw if w[2] is not None]
        out += [f"Log windows that contain an epoch boundary (evaluation + checkpoint hand-off inside): "
                f"{len(bw)}; host wall time {min(r):.2f}x-{max(r):.2f}x (median {statistics.median(r):.2f}x) "
                f"of a steady window.", ""]
    if epochs:
        out += ["| epoch | end-to-end img/s | % of steady | wall s | evaluate ms | checkpoint hand-off ms | "
                "previous write (background) ms | its phases (ms) |", "|---:|---:|---:|---:|---:|---:|---:|---|"]
        for e, rate, wall, ev, ck, wr, parts in epochs:
            out.append(f"| {int(e)} | {rate:,.1f} | {100 * rate / st_rate:.1f} % | {wall:.3f} | {ev:.1f} | "
                       f"{ck:.1f} | {wr:.1f} | {parts} |")
        later = [x[1] for x in epochs[1:]] or [epochs[0][1]]
        out += ["", f"Epochs after the first (graph capture is in epoch 0): median end to end "
                    f"**{statistics.median(later):,.1f} img/s = {100 * statistics.median(later) / st_rate:.1f} %** "
                    f"of the steady step rate."]
    if run:
        out += ["", f"Whole run: {run[0]:,.1f} img/s end to end over {run[1]} steps ({run[2]:.2f} s incl. graph "
                    f"capture, evaluation, checkpoints) = {100 * run[0] / st_rate:.1f} % of the steady step rate."]
    print("\n".join(out))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None))
