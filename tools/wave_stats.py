"""Heavy stage in wave mode (csrc/wave.hip) on a generated configuration:
heavy histories, DFS iterations per history (max / mean; the DFS runs
the histories whose state DAG does not fit), the DAG's share and the call's
device time, over a few calls (diagnostic; the wave_stats_ptr knob).
    python tools/wave_stats.py bank_4x16 1000000 [knob=value ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402


def main():
    name, n = sys.argv[1], int(sys.argv[2])
    nostats = "--nostats" in sys.argv          # device times only (the timers cost the DAG's levels time)
    ctx = device.Context(0)
    params = dict(kv.split("=") for kv in sys.argv[3:] if kv != "--nostats")
    ctx.set_param("heavy_mode", 0)
    for k, v in params.items():
        ctx.set_param(k, int(v))
    dev = torch.device("cuda:0")
    stats = torch.zeros(16, dtype=torch.int64, device=dev)
    if not nostats:
        ctx.set_param("wave_stats_ptr", stats.data_ptr())
    hdr, ev, _ = gen.generate_config(name, 0, n, threads=16)
    d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    d_st = torch.empty(n, dtype=torch.uint8, device=dev)
    d_nd = torch.empty(n, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for i in range(8 if nostats else 5):
        stats.zero_()
        ctx.timing_reset()
        ctx.check_device(gen.CONFIGS[name]["model_id"], d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev),
                         d_st.data_ptr(), d_nd.data_ptr(), stream=s)
        torch.cuda.synchronize()
        q = stats.cpu().numpy()
        probe = ctx.probe()
        heavy = probe["heavy32"] + probe["heavy64"]
        s0, call = ctx.timing_read()
        if nostats:
            print(f"call {i}: device {call[0]:.3f} ms (stage 0 {s0[0]:.3f}); heavy histories {heavy}", flush=True)
            continue
        print(f"call {i}: device {call[0]:.3f} ms (stage 0 {s0[0]:.3f}); heavy histories {heavy}, "
              f"DFS iterations max {q[0]}, mean {q[1] / max(heavy, 1):.1f}; cycles per history max {q[2]}, "
              f"mean {q[3] / max(heavy, 1):.0f}; cycles per iteration {q[3] / max(q[1], 1):.0f}; "
              f"nodes per history {q[4] / max(heavy, 1):.1f}; state DAG: {q[5]} histories, cycles max {q[6]} "
              f"mean {q[7] / max(q[5], 1):.0f}; per DAG history: levels {q[13] / max(q[5], 1):.1f}, cycles in "
              f"state lanes {q[8] / max(q[5], 1):.0f}, item step {q[9] / max(q[5], 1):.0f}, "
              f"dedup {q[10] / max(q[5], 1):.0f}, backward {q[11] / max(q[5], 1):.0f}, tail {q[12] / max(q[5], 1):.0f}",
              flush=True)
    ctx.set_param("wave_stats_ptr", 0)
    ctx.close()


if __name__ == "__main__":
    main()
