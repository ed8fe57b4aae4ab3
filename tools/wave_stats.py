"""Wave-stage diagnostics on a generated configuration: histories, DFS
iterations (wavefront ticks) and s_memtime cycles per history."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402


def main():
    name, n = sys.argv[1], int(sys.argv[2])
    ctx = device.Context(0)
    params = dict(kv.split("=") for kv in sys.argv[3:])
    for k, v in params.items():
        ctx.set_param(k, int(v))
    dev = torch.device("cuda:0")
    grid = int(params.get("wave_grid", 0)) or 3 * torch.cuda.get_device_properties(0).multi_processor_count
    stats = torch.zeros(grid * 8, dtype=torch.int64, device=dev)
    ctx.set_param("wave_stats_ptr", stats.data_ptr())
    ctx.set_param("heavy_mode", 0)
    hdr, ev, _ = gen.generate_config(name, 0, n, threads=16)
    d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    d_st = torch.empty(n, dtype=torch.uint8, device=dev)
    d_nd = torch.empty(n, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for i in range(3):
        stats.zero_()
        ctx.check_device(gen.CONFIGS[name]["model_id"], d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev),
                         d_st.data_ptr(), d_nd.data_ptr(), stream=s)
        torch.cuda.synchronize()
        q = stats.view(-1, 8).cpu().numpy()
        h = q[:, 0].sum()
        print(f"call {i}: {ctx.last_kernel_ms():.3f} ms; wave histories {h}, ticks/hist {q[:, 1].sum() / max(h, 1):.1f}"
              f" (max {q[:, 4].max()}), cycles/tick {q[:, 2].sum() / max(q[:, 1].sum(), 1):.0f}, "
              f"splits/hist {q[:, 3].sum() / max(h, 1):.1f}, nodes/hist {q[:, 7].sum() / max(h, 1):.1f}, "
              f"busiest wave {q[:, 2].max() / 2.4e3:.1f} us (s_memtime at ~100MHz? raw {q[:, 2].max()})", flush=True)
    ctx.set_param("wave_stats_ptr", 0)


if __name__ == "__main__":
    main()
