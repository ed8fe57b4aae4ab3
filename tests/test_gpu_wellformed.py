"""GPU parity of the batched `wellformed` kernel (csrc/wellformed.hip)
against the literal restatement oracle/wellformed_ref.py and the host mirror
qsmd.wellformed (src/Linearisability.hs:97-135)."""

import random

import numpy as np
import pytest

import histgen
import wellformed_ref
from qsmd import codec, gen
from qsmd.linearisability import wellformed, wellformed_batch

pytestmark = pytest.mark.gpu


def _as_tuple(err):
    return None if err is None else (err.kind, tuple(err.args))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_wellformed_any_shape(ctx, seed):
    rng = random.Random(seed)
    hs = []
    for _ in range(3000):
        n_pid = rng.randint(1, 6)
        if rng.random() < 0.5:
            hs.append(histgen.random_history(rng, rng.choice(["bank", "ticket"]), rng.randint(0, 40), n_pid))
        else:
            hs.append(histgen.wellformed_history(rng, rng.choice(["bank", "ticket"]), rng.randint(0, 20), n_pid))
    pid_lists = [["p0", "p1", "p2", "p3", "p4", "p5"], ["p3", "p1"], ["p5", "p4", "p3", "p2", "p1", "p0"],
                 ["p2"], ["nobody", "p0"]]
    for pids in pid_lists:
        got = wellformed_batch(pids, hs, ctx=ctx)
        for h, g in zip(hs, got):
            ref = wellformed_ref.wellformed(pids, h)
            assert _as_tuple(g) == ref, (pids, h, g, ref)
            assert _as_tuple(wellformed(pids, h)) == ref


def test_wellformed_long_and_many_pids(ctx):
    rng = random.Random(9)
    hs = [histgen.random_history(rng, "ticket", rng.randint(60, 128), rng.randint(20, 100)) for _ in range(500)]
    hs += [histgen.wellformed_history(rng, "bank", 64, 90, p_pending=0.0)[:128] for _ in range(200)]
    pids = [f"p{i}" for i in range(100)]
    got = wellformed_batch(pids, hs, ctx=ctx)
    for h, g in zip(hs, got):
        assert _as_tuple(g) == wellformed_ref.wellformed(pids, h)


def test_wellformed_encode_errors(ctx):
    hdr = np.zeros(3, dtype=codec.HDR_DTYPE)
    ev = np.zeros(4, dtype=codec.EV_DTYPE)
    hdr[0] = (0, 200, 1, 0, 0, 0)           # too many events / beyond the buffer
    hdr[1] = (0, 2, 1, 0, 0, 0)             # pid 3 >= n_pid
    ev[1]["kp"] = 3
    hdr[2] = (2, 2, 1, 0, 0, 0)             # fine: L R of pid 0
    ev[3]["kp"] = 0x80
    out = ctx.wellformed_arrays(hdr, ev)
    assert list(out["code"]) == [codec.WF_ENCODE_ERROR, codec.WF_ENCODE_ERROR, 0]


def test_wellformed_full_size_device(ctx):
    """Config 2 at full size through the device entry point: every generated
    history is per-client sequential (size-independent property)."""
    torch = pytest.importorskip("torch")
    n = 1_000_000
    hdr, ev, _ = gen.generate_config("bank_4x16", 0, n)
    dev = torch.device("cuda:0")
    d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    d_out = torch.zeros(n * 8, dtype=torch.uint8, device=dev)
    ctx.wellformed_device(d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev), d_out.data_ptr(),
                          stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy().view(codec.WF_DTYPE)
    assert (out["code"] == 0).all()
    # break one history in a known way: swap its first invocation and response
    ev2 = ev.copy()
    o = int(hdr[777]["ev_off"])
    first_r = o + int(np.nonzero(ev2["kp"][o:o + 32] & 0x80)[0][0])
    ev2[[o, first_r]] = ev2[[first_r, o]]
    out2 = ctx.wellformed_arrays(hdr[770:780], ev2)
    assert (out2["code"][[0, 1, 2, 3, 4, 5, 6, 8, 9]] == 0).all() and out2["code"][7] != 0
