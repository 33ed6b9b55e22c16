"""Occupancy timeline of one k_trace launch from a per-wave dump.

The dump (TPT_DEBUG_WAVES=<file> with a TPT_PROFILE_PHASES build) holds 8 u64 per
wave: start tick, life, traversal steps, shading passes, rays, 4-wide visits,
the heaviest lane's rays, shading-pass ticks (s_memrealtime, 100 MHz).

Prints how long the launch ran with the chip full (live waves >= the resident
capacity) and the tail: the time from the last wave start to the launch end,
and the wave-time the chip could have held but did not (idle slot fraction).
Usage: python tools/wave_timeline.py dump.bin [capacity=5120]
"""
import sys

import numpy as np


def main():
    d = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8).astype(np.float64)
    cap = int(sys.argv[2]) if len(sys.argv) > 2 else 5120
    d = d[d[:, 1] > 0]
    t0 = d[:, 0].min()
    start = (d[:, 0] - t0) / 100.0   # us
    end = start + d[:, 1] / 100.0
    span = end.max()
    ev = np.concatenate([np.stack([start, np.ones_like(start)], 1), np.stack([end, -np.ones_like(end)], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    live = np.cumsum(ev[:, 1])
    dt = np.diff(np.append(ev[:, 0], span))
    busy = np.minimum(live, cap)
    util = float((busy * dt).sum() / (cap * span))
    full = float(dt[live >= cap * 0.98].sum())
    last_start = start.max()
    life = d[:, 1] / 100.0
    order = np.argsort(-life)
    print(f"waves {len(d)}  launch {span / 1000:.2f} ms  slot utilisation {util:.3f}  "
          f"chip-full {full / 1000:.2f} ms  last start {last_start / 1000:.2f} ms  "
          f"tail after last start {(span - last_start) / 1000:.2f} ms")
    print(f"wave life ms: mean {life.mean() / 1000:.2f}  median {np.median(life) / 1000:.2f}  "
          f"p99 {np.percentile(life, 99) / 1000:.2f}  max {life.max() / 1000:.2f}")
    for q in (0.5, 0.75, 0.9, 0.95, 0.99):
        # time at which the live count first drops below q*cap for good
        below = np.nonzero(live < q * cap)[0]
        above = np.nonzero(live >= q * cap)[0]
        t = ev[above[-1] + 1, 0] if len(above) and above[-1] + 1 < len(ev) else span
        print(f"  live < {q:.2f}*cap from {t / 1000:.2f} ms ({(span - t) / span * 100:.1f} % of the launch)")
    print("heaviest waves (start ms, life ms, rays, wide, max lane rays):")
    for i in order[:5]:
        print(f"  {start[i] / 1000:8.2f} {life[i] / 1000:8.2f} {int(d[i, 4]):10d} {int(d[i, 5]):10d} {int(d[i, 6]):8d}")


if __name__ == "__main__":
    main()
