"""Randomised parity sweep on the GPU (tools/stress_parity.py): generated
batches with random generator parameters and random any-shape histories (up
to 100 events / 12 pids), with random stage budgets, heavy-stage modes, memo
table sizes and giant-stage budgets per batch, against the C oracle --
statuses, node counts and witnesses.  The sweep that found the Map.!
descent in the heavy stage (tests/golden/wave_model_error_case.npz); a
bounded slice of it runs here (the full sweeps: profiles/r02/stress_parity.json)."""

import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))


@pytest.mark.parametrize("seed", [31, 32])
def test_random_knobs_and_shapes(ctx, seed):
    import stress_parity
    stats = stress_parity.run(ctx, batches=60, seed=seed, knobs=True, wide=True)
    assert stats["histories"] > 0
    assert stats["mismatch_status"] == stats["mismatch_nodes"] == stats["mismatch_witness"] == 0, stats
    # (the context's 60 s time limit never fires here: every batch is compared in full)
    assert stats["timed_out_batches"] == 0, stats
