"""The SchedulerHistory wire format (src/Scheduler.hs:69-72, sent at :204-205)
-> histories -> the SoA batch (qsmd/wire.py).

Parity unpinned: there is no GHC here to produce reference bytes.  The
byte strings below are written out by hand from the documented `binary`
rules (qsmd/wire.py docstring), independently of the module's encoder, for
the reference's own example history (KAT-2, test/TicketDispenser.hs:326-347)
and the Bank KAT-7; the decoded batches must check exactly as the KATs.
"""

import random
import struct

import numpy as np
import pytest

import oracle_c
from kats import KATS
from qsmd import codec, gen, models, wire

NODE = b"127.0.0.1:10501:0"                      # an EndPointAddress of the reference's TCP transport


def pid_bytes(counter, unique=0, addr=NODE):
    return struct.pack(">q", len(addr)) + addr + struct.pack(">ii", unique, counter)


def i64(v):
    return struct.pack(">q", v)


def small_integer(v):
    return b"\x00" + struct.pack(">i", v)


# KAT-2 by hand: every event on the test process's pid (quirk Q1)
P8 = pid_bytes(8)
KAT2_BYTES = (i64(6)
              + P8 + b"\x00" + b"\x01"                 # Left Reset
              + P8 + b"\x01" + b"\x01"                 # Right Ok
              + P8 + b"\x00" + b"\x00"                 # Left TakeTicket
              + P8 + b"\x00" + b"\x00"                 # Left TakeTicket
              + P8 + b"\x01" + b"\x00" + i64(2)        # Right (Number 2)
              + P8 + b"\x01" + b"\x00" + i64(1))       # Right (Number 1)

PA, PB = pid_bytes(11), pid_bytes(12)
KAT7_BYTES = (i64(10)
              + PA + b"\x00" + b"\x00" + PA                          # a: Left (OpenAccount a)
              + PA + b"\x01" + b"\x00"                               # a: Right AccountCreated
              + PB + b"\x00" + b"\x00" + PB                          # b: Left (OpenAccount b)
              + PB + b"\x01" + b"\x00"                               # b: Right AccountCreated
              + PB + b"\x00" + b"\x01" + PB + small_integer(10)      # b: Left (Deposit b 10)
              + PB + b"\x01" + b"\x01"                               # b: Right DepositMade
              + PA + b"\x00" + b"\x03" + PA                          # a: Left (CheckBalance a)
              + PB + b"\x00" + b"\x04" + PB + small_integer(5) + PA  # b: Left (Transfer b 5 a)
              + PA + b"\x01" + b"\x07" + small_integer(3)            # a: Right (Balance 3)
              + PB + b"\x01" + b"\x03")                              # b: Right TransferMade


def _same_batch(b1, b2):
    assert np.array_equal(b1.hdr[["n_ev", "n_pid", "model_id"]], b2.hdr[["n_ev", "n_pid", "model_id"]])
    assert np.array_equal(b1.events, b2.events)


def test_kat2_bytes_decode_to_the_reference_example():
    h = wire.decode_scheduler_history(KAT2_BYTES, models.MODEL_TICKET)
    m, ref, status, nodes = KATS["KAT2_reference_example"]
    assert [ev for _, ev in h] == [ev for _, ev in ref]
    assert len({p for p, _ in h}) == 1 and str(h[0][0]).endswith(":8")
    _same_batch(wire.decode_batch([KAT2_BYTES], models.MODEL_TICKET), codec.encode(models.TICKET, [ref]))
    assert wire.encode_scheduler_history(h, models.MODEL_TICKET) == KAT2_BYTES
    st, nd, _ = oracle_c.check_batch(models.MODEL_TICKET, *wire.batch_arrays([KAT2_BYTES], models.MODEL_TICKET))
    assert (codec.STATUS_NAMES[int(st[0])], int(nd[0])) == (status, nodes)


def test_kat7_bytes_decode_to_the_bank_kat():
    h = wire.decode_scheduler_history(KAT7_BYTES, models.MODEL_BANK)
    _, ref, status, nodes = KATS["KAT7_bank_concurrent"]
    # the reference's Bank accounts are the pids themselves (test/Bank.hs:54-60)
    rename = {"a": h[0][0], "b": h[2][0]}

    def ren(ev):
        kind, x = ev
        if kind == "L":
            return (kind, tuple(rename.get(v, v) if isinstance(v, str) and v in rename else v for v in x))
        return ev
    assert h == [(rename[p], ren(ev)) for p, ev in ref]
    assert wire.encode_scheduler_history(h, models.MODEL_BANK) == KAT7_BYTES
    _same_batch(wire.decode_batch([KAT7_BYTES], models.MODEL_BANK), codec.encode(models.BANK, [ref]))
    st, nd, _ = oracle_c.check_batch(models.MODEL_BANK, *wire.batch_arrays([KAT7_BYTES], models.MODEL_BANK))
    assert (codec.STATUS_NAMES[int(st[0])], int(nd[0])) == (status, nodes)


def test_large_integers_are_encode_errors_not_wrong_answers():
    # Deposit b (2^40): binary's big-Integer form (tag 1, sign, LE magnitude bytes)
    big = b"\x01" + b"\x01" + i64(6) + (2 ** 40).to_bytes(6, "little")
    neg = b"\x01" + b"\xff" + i64(5) + (2 ** 33).to_bytes(5, "little")
    hb = i64(2) + PB + b"\x00" + b"\x01" + PB + big + PB + b"\x01" + b"\x01"
    hn = i64(2) + PB + b"\x00" + b"\x02" + PB + neg + PB + b"\x01" + b"\x06"
    assert wire.decode_scheduler_history(hb, models.MODEL_BANK)[0][1] == ("L", ("Deposit", wire.ProcessId(NODE, 0, 12), 2 ** 40))
    assert wire.decode_scheduler_history(hn, models.MODEL_BANK)[0][1][1][2] == -(2 ** 33)
    for h in (hb, hn):
        b = wire.decode_batch([h, KAT7_BYTES], models.MODEL_BANK)
        assert b.hdr["model_id"][0] == codec.BAD_MODEL and b.hdr["model_id"][1] == models.MODEL_BANK
        w = wire.Writer()
        w.integer(2 ** 40 if h is hb else -(2 ** 33))
        assert w.bytes() == (big if h is hb else neg)


@pytest.mark.parametrize("name", ["ticket_2x10", "bank_4x16_bugs", "bank_6x24"])
def test_round_trip_generated_histories(name):
    """Generated batches -> histories with ProcessIds -> wire bytes -> the same
    batch (pids and accounts renumbered identically)."""
    hdr, ev, _ = gen.generate_config(name, 3, 300)
    mid = gen.CONFIGS[name]["model_id"]
    m = models.BY_ID[mid]
    shape = codec.Batch(m, hdr, ev, [{i: i for i in range(int(h["n_pid"]))} for h in hdr],
                        [{i: i for i in range(8)} for _ in hdr])
    rng = random.Random(name)
    payloads = []
    for i in range(len(hdr)):
        pmap = {p: wire.ProcessId(NODE, rng.randrange(2 ** 31), 100 + p) for p in range(16)}
        h = codec.decode_history(shape, i)
        h = [(pmap[p], (k, tuple(pmap[v] if j in ((1,) if x[0] != "Transfer" else (1, 3)) else v
                                 for j, v in enumerate(x)) if (k == "L" and isinstance(x, tuple)) else x))
             for p, (k, x) in h]
        payloads.append(wire.encode_scheduler_history(h, mid))
    b = wire.decode_batch(payloads, mid)
    st1, nd1, _ = oracle_c.check_batch(mid, hdr, ev, threads=4, max_nodes=10**7)
    st2, nd2, _ = oracle_c.check_batch(mid, b.hdr, b.events, threads=4, max_nodes=10**7)
    assert np.array_equal(st1, st2) and np.array_equal(nd1, nd2)


def test_malformed_bytes_raise():
    for bad in (KAT2_BYTES[:-1],                         # truncated
                KAT2_BYTES + b"\x00",                    # trailing byte
                i64(1) + P8 + b"\x02" + b"\x00",         # Either tag 2
                i64(1) + P8 + b"\x00" + b"\x05",         # Request tag 5
                i64(2 ** 40)):                           # absurd length
        with pytest.raises(wire.WireError):
            wire.decode_scheduler_history(bad, models.MODEL_TICKET)
    with pytest.raises(wire.WireError):
        wire.decode_scheduler_history(i64(1) + PA + b"\x01" + b"\x08", models.MODEL_BANK)   # BankResponse tag 8
