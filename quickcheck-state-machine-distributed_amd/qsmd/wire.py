"""The reference's history wire format -> histories -> the SoA batch.

The reference's scheduler ends a run by sending the supervisor
``SchedulerHistory hist`` (``src/Scheduler.hs:204-205``), a
``newtype SchedulerHistory pid inv resp = SchedulerHistory (History pid inv resp)``
with a Generic-derived ``Binary`` instance (``src/Scheduler.hs:69-72``); the
history is ``[(pid, Either inv resp)]`` (``src/Linearisability.hs:18``) with
``pid = ProcessId`` and the models' own Generic ``Binary`` instances
(``test/Bank.hs:44-73``, ``test/TicketDispenser.hs:51-63``).  This module
decodes those payload bytes (and encodes them, for tests) so a non-Haskell
consumer can feed real scheduler output to the checker.

Encoding rules restated from ``binary`` 0.8.5.1 and ``distributed-process``
0.7.3 / ``network-transport`` 0.5 as pinned by the reference's Stackage
snapshot lts-11.2 (``stack.yaml:1-7``), neither of which is vendored:

* ``Int`` = 8 bytes big-endian two's complement; ``Int32`` = 4 bytes BE;
* a list = its length as ``Int``, then the elements; a pair = both fields;
* ``Either`` = tag byte 0 (``Left``) / 1 (``Right``), then the payload;
* a Generic sum type with at most 256 constructors = one tag byte holding the
  constructor's index in declaration order, then its fields in order; a
  single-constructor type (the newtype) has no tag;
* ``Integer`` = tag byte 0 + ``Int32`` BE when the value fits in Int32,
  else tag byte 1, a sign byte (1 = positive, 255 = negative), and the
  magnitude's bytes least significant first as a ``[Word8]``;
* ``ProcessId`` = its ``NodeId`` (the ``EndPointAddress``: a strict
  ``ByteString`` = length as ``Int`` + bytes) then its ``LocalProcessId``
  (``lpidUnique``, ``lpidCounter``: two ``Int32``).

Parity unpinned: no GHC exists in this image or on the GPU box, so no byte
string produced by the reference itself pins these rules; the tests check
hand-built byte strings of the KAT histories against them
(``tests/test_wire.py``).
"""

from __future__ import annotations

import struct
from typing import NamedTuple

import numpy as np

from . import codec, models


class WireError(ValueError):
    """The bytes are not a well-formed SchedulerHistory encoding."""


class ProcessId(NamedTuple):
    """distributed-process ``ProcessId``: node address + local id."""
    address: bytes
    unique: int
    counter: int

    def __str__(self):                      # Show ProcessId: pid://<address>:<counter>
        return f"pid://{self.address.decode('latin-1')}:{self.counter}"


class Reader:
    def __init__(self, data: bytes, pos: int = 0):
        self.data = memoryview(data)
        self.pos = pos

    def take(self, n: int) -> bytes:
        if n < 0 or self.pos + n > len(self.data):
            raise WireError(f"truncated: need {n} bytes at offset {self.pos}")
        b = bytes(self.data[self.pos:self.pos + n])
        self.pos += n
        return b

    def word8(self) -> int:
        return self.take(1)[0]

    def int32(self) -> int:
        return struct.unpack(">i", self.take(4))[0]

    def int64(self) -> int:
        return struct.unpack(">q", self.take(8))[0]

    def length(self) -> int:
        n = self.int64()
        if n < 0 or n > len(self.data) - self.pos:     # every element takes >= 1 byte
            raise WireError(f"bad list length {n} at offset {self.pos - 8}")
        return n

    def bytestring(self) -> bytes:
        return self.take(self.length())

    def integer(self) -> int:
        tag = self.word8()
        if tag == 0:
            return self.int32()
        if tag != 1:
            raise WireError(f"bad Integer tag {tag}")
        sign = self.word8()
        if sign not in (1, 255):
            raise WireError(f"bad Integer sign byte {sign}")
        mag = self.take(self.length())
        v = int.from_bytes(mag, "little")
        return v if sign == 1 else -v

    def process_id(self) -> ProcessId:
        addr = self.bytestring()
        return ProcessId(addr, self.int32(), self.int32())

    def tag(self, n: int, what: str) -> int:
        t = self.word8()
        if t >= n:
            raise WireError(f"bad {what} constructor tag {t}")
        return t


class Writer:
    def __init__(self):
        self.parts = []

    def bytes(self) -> bytes:
        return b"".join(self.parts)

    def word8(self, v):
        self.parts.append(bytes([v]))

    def int32(self, v):
        self.parts.append(struct.pack(">i", v))

    def int64(self, v):
        self.parts.append(struct.pack(">q", v))

    def bytestring(self, b):
        self.int64(len(b))
        self.parts.append(bytes(b))

    def integer(self, v):
        if -2 ** 31 <= v < 2 ** 31:
            self.word8(0)
            self.int32(v)
        else:
            self.word8(1)
            self.word8(1 if v > 0 else 255)
            mag = abs(v).to_bytes((abs(v).bit_length() + 7) // 8, "little")
            self.int64(len(mag))
            self.parts.append(mag)

    def process_id(self, p: ProcessId):
        self.bytestring(p.address)
        self.int32(p.unique)
        self.int32(p.counter)


# ---------------------------------------------------------------- the models
# Constructor order of the Haskell declarations = the tag byte.

TICKET_REQ = ("TakeTicket", "Reset")                       # test/TicketDispenser.hs:51-54
TICKET_RESP = ("Number", "Ok")                             # :59-62
BANK_REQ = ("OpenAccount", "Deposit", "Withdraw", "CheckBalance", "Transfer")   # test/Bank.hs:44-50
BANK_RESP = ("AccountCreated", "DepositMade", "WithdrawalMade", "TransferMade",  # :66-73
             "AccountAlreadyExists", "AccountDoesntExist", "InsufficientFunds", "Balance")


def _ticket_inv(r):
    return TICKET_REQ[r.tag(2, "Request")]


def _ticket_resp(r):
    t = r.tag(2, "Response")
    return ("Number", r.int64()) if t == 0 else "Ok"


def _bank_inv(r):
    op = BANK_REQ[r.tag(5, "BankRequestF")]
    if op in ("OpenAccount", "CheckBalance"):
        return (op, r.process_id())
    if op in ("Deposit", "Withdraw"):
        return (op, r.process_id(), r.integer())
    return (op, r.process_id(), r.integer(), r.process_id())


def _bank_resp(r):
    t = r.tag(8, "BankResponse")
    return ("Balance", r.integer()) if t == 7 else BANK_RESP[t]


def _put_ticket_inv(w, inv):
    w.word8(TICKET_REQ.index(inv))


def _put_ticket_resp(w, resp):
    if resp == "Ok":
        w.word8(1)
    else:
        w.word8(0)
        w.int64(resp[1])


def _put_bank_inv(w, req):
    w.word8(BANK_REQ.index(req[0]))
    w.process_id(req[1])
    if req[0] in ("Deposit", "Withdraw", "Transfer"):
        w.integer(req[2])
    if req[0] == "Transfer":
        w.process_id(req[3])


def _put_bank_resp(w, resp):
    if isinstance(resp, tuple):
        w.word8(7)
        w.integer(resp[1])
    else:
        w.word8(BANK_RESP.index(resp))


CODECS = {
    models.MODEL_TICKET: (_ticket_inv, _ticket_resp, _put_ticket_inv, _put_ticket_resp),
    models.MODEL_BANK: (_bank_inv, _bank_resp, _put_bank_inv, _put_bank_resp),
}


def decode_scheduler_history(data: bytes, model_id: int, pos: int = 0, with_end: bool = False):
    """One ``SchedulerHistory ProcessId inv resp`` payload -> a history
    ``[(ProcessId, ("L", inv) | ("R", resp))]`` in the shapes of qsmd.models."""
    get_inv, get_resp, _, _ = CODECS[model_id]
    r = Reader(data, pos)
    out = []
    for _ in range(r.length()):
        pid = r.process_id()
        side = r.word8()
        if side == 0:
            out.append((pid, ("L", get_inv(r))))
        elif side == 1:
            out.append((pid, ("R", get_resp(r))))
        else:
            raise WireError(f"bad Either tag {side}")
    if with_end:
        return out, r.pos
    if r.pos != len(r.data):
        raise WireError(f"{len(r.data) - r.pos} trailing bytes")
    return out


def encode_scheduler_history(history, model_id: int) -> bytes:
    """The inverse of decode_scheduler_history (pids must be ProcessIds)."""
    _, _, put_inv, put_resp = CODECS[model_id]
    w = Writer()
    w.int64(len(history))
    for pid, (kind, x) in history:
        w.process_id(pid)
        if kind == "L":
            w.word8(0)
            put_inv(w, x)
        else:
            w.word8(1)
            put_resp(w, x)
    return w.bytes()


def decode_batch(payloads, model_id: int, model0=None) -> codec.Batch:
    """Many SchedulerHistory payloads -> one SoA batch (include/qsmd.h).
    A payload that is not a well-formed encoding raises WireError; a history
    whose values fall outside the batch encoding (Integer beyond Int32, > 8
    Bank accounts, > 128 events or pids) becomes an ENCODE_ERROR entry, as
    codec.encode does."""
    hs = [decode_scheduler_history(p, model_id) for p in payloads]
    return codec.encode(models.BY_ID[model_id], hs, model0)


def batch_arrays(payloads, model_id: int):
    """(hdr, events) numpy arrays of decode_batch, for the C ABI."""
    b = decode_batch(payloads, model_id)
    return np.ascontiguousarray(b.hdr), np.ascontiguousarray(b.events)
