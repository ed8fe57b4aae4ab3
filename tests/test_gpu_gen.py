"""On-device history generation (csrc/gen.hip, qsmd_gen_batch_device):
byte-identical to the host generator (csrc/gen/gen.cpp) for every BASELINE
config and the generator's other policies, at any first index and ev_base."""

import numpy as np
import pytest

from qsmd import codec, gen

pytestmark = pytest.mark.gpu

CASES = [(name, {}) for name in gen.CONFIGS] + [
    ("bank_4x16", {"lin_policy": 0}), ("bank_4x16", {"p_bug": 1.0, "money_max": 7}),
    ("ticket_2x10", {"pid_mode": 0, "p_bug": 0.7}), ("bank_6x24", {"overlap": 0, "n_clients": 8, "n_ops": 64}),
    ("ticket_8x64", {"p_bug": 0.3, "overlap": 3}), ("bank_4x16", {"n_clients": 1, "n_ops": 5, "prefix_ops": 0}),
]


@pytest.mark.parametrize("name,override", CASES)
@pytest.mark.parametrize("first,ev_base", [(0, 0), (123457, 1000)])
def test_device_generator_matches_host(ctx, name, override, first, ev_base):
    torch = pytest.importorskip("torch")
    kw = dict(gen.CONFIGS[name])
    kw.update(override)
    p = gen.params(**kw)
    n = 20000
    per = 2 * p.n_ops
    hdr = np.zeros(n, dtype=codec.HDR_DTYPE)
    ev = np.zeros(n * per, dtype=codec.EV_DTYPE)
    bug = np.zeros(n, dtype=np.uint8)
    assert gen._load().qsmd_gen_batch(p, first, n, ev_base, hdr.ctypes.data, ev.ctypes.data, bug.ctypes.data, 8) == 0
    dev = torch.device("cuda:0")
    d_hdr = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_ev = torch.zeros(n * per * 8, dtype=torch.uint8, device=dev)
    d_bug = torch.zeros(n, dtype=torch.uint8, device=dev)
    ctx.gen_device(p, first, n, d_hdr.data_ptr(), d_ev.data_ptr(), d_bug.data_ptr(), ev_base=ev_base,
                   stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(d_hdr.cpu().numpy(), hdr.view(np.uint8))
    assert np.array_equal(d_ev.cpu().numpy(), ev.view(np.uint8))
    assert np.array_equal(d_bug.cpu().numpy(), bug)
    if kw.get("p_bug", 0) > 0:
        assert 0 < bug.sum() < n or kw["p_bug"] == 1.0


def test_device_generator_rejects_bad_params(ctx):
    from qsmd import device
    p = gen.params(**gen.CONFIGS["bank_4x16"])
    p.n_clients = 9
    with pytest.raises(device.DeviceError):
        ctx.gen_device(p, 0, 10, 0, 0)
