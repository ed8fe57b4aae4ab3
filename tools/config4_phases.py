"""BASELINE config 4 through the host entry with the wave-mode diagnostic
counters (wave_stats_ptr): the state DAG's cycles per phase and level
(diagnostic; the timers themselves cost time).
    python tools/config4_phases.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402


def main():
    h, e, _ = gen.adversarial_ticket(8, 64, bug=True)
    ctx = device.Context(0)
    stats = torch.zeros(16, dtype=torch.int64, device="cuda:0")
    ctx.set_param("wave_stats_ptr", stats.data_ptr())
    flags = device.QSMD_FLAG_EXHAUSTIVE | device.QSMD_FLAG_MEMO
    for mode, fl in (("memo", flags), ("exhaustive", device.QSMD_FLAG_EXHAUSTIVE)):
        for _ in range(3):
            stats.zero_()
            st, nd, _, _ = ctx.check_arrays(1, h, e, flags=fl)
        q = stats.cpu().numpy()
        n = max(int(q[5]), 1)
        lv = q[13] / n
        print(f"{mode}: status {int(st[0])} nodes {int(nd[0])}; DAG histories {q[5]}, cycles {q[7] / n:.0f}, "
              f"levels {lv:.0f}; per level: state lanes {q[8] / n / lv:.0f}, item step {q[9] / n / lv:.0f}, "
              f"dedup {q[10] / n / lv:.0f}, backward {q[11] / n / lv:.0f}; tail {q[12] / n:.0f}", flush=True)
    ctx.set_param("wave_stats_ptr", 0)
    ctx.close()


if __name__ == "__main__":
    main()
