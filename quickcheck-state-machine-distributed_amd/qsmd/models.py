"""Device models: the user closures the reference passes to ``linearisable``.

The reference's search calls only the model closures its callers pass
(``src/Linearisability.hs:52-58``).  On the GPU those closures are compiled
device functors (``csrc/models.hip``); this module is their host side:

* the constructor <-> code tables of include/qsmd.h,
* the Haskell model functions themselves (used on the host for ``trace``
  printing and witness replay, never for the search),
* ``init_model`` and the packing of a non-default ``model0``.

Values use the same shapes as the Haskell constructors:

TicketDispenser (test/TicketDispenser.hs:51-102)
    inv  ``'TakeTicket' | 'Reset'``
    resp ``('Number', i) | 'Ok'``
    model ``None`` (Nothing) | ``int`` (Just n)

Bank (test/Bank.hs:41-131)
    inv  ``('OpenAccount', a) | ('Deposit', a, m) | ('Withdraw', a, m)
         | ('CheckBalance', a) | ('Transfer', a, m, b)``
    resp ``'AccountCreated' | 'DepositMade' | 'WithdrawalMade' |
         'TransferMade' | 'AccountAlreadyExists' | 'AccountDoesntExist' |
         'InsufficientFunds' | ('Balance', v)``
    model ``dict`` account -> int (Data.Map, treated as immutable)
"""

from __future__ import annotations

import ctypes

MODEL_TICKET = 1
MODEL_BANK = 2

I32_MIN, I32_MAX = -(2 ** 31), 2 ** 31 - 1
BANK_MAX_ACCOUNTS = 8


class ModelError(Exception):
    """The reference model raises (Haskell exception), e.g. ``Map.!`` on a
    missing account in Bank's ``post`` (test/Bank.hs:128)."""


class EncodeError(ValueError):
    """A value cannot be represented in the include/qsmd.h encoding."""


def _i32(v):
    if not isinstance(v, int) or isinstance(v, bool) or not (I32_MIN <= v <= I32_MAX):
        raise EncodeError(f"value {v!r} outside int32")
    return v


class DeviceModel:
    """Host half of a device functor pair (transition, postcondition)."""

    name = ""
    model_id = 0

    # -- Haskell semantics (host replay / trace only) ---------------------
    @staticmethod
    def transition(model, ev):
        raise NotImplementedError

    @staticmethod
    def postcondition(model, inv, resp):
        raise NotImplementedError

    init_model = None

    # -- encoding ----------------------------------------------------------
    def new_account_map(self, model0):
        return {}

    def encode_inv(self, inv, accounts):
        raise NotImplementedError

    def encode_resp(self, resp):
        raise NotImplementedError

    def pack_model0(self, model0, accounts):
        """Return a ctypes struct for ``model0`` or None for init_model."""
        raise NotImplementedError

    def show_model(self, model):
        return repr(model)

    def show_inv(self, inv):
        return repr(inv)

    def show_resp(self, resp):
        return repr(resp)


# ---------------------------------------------------------------------------
# TicketDispenser
# ---------------------------------------------------------------------------

class TicketModel(ctypes.Structure):
    _fields_ = [("is_just", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("n", ctypes.c_int64)]


class TicketDispenser(DeviceModel):
    name = "ticket"
    model_id = MODEL_TICKET
    init_model = None                               # Nothing

    INV = {"TakeTicket": 0, "Reset": 1}
    INV_NAMES = {v: k for k, v in INV.items()}

    @staticmethod
    def transition(m, ev):                          # TicketDispenser.hs:81-85
        kind, x = ev
        if kind == "R":
            return m
        if x == "TakeTicket":
            return None if m is None else m + 1
        return 0

    @staticmethod
    def postcondition(m, inv, resp):                # TicketDispenser.hs:99-102
        if inv == "TakeTicket" and isinstance(resp, tuple) and resp[0] == "Number":
            return m is not None and resp[1] == m + 1
        return inv == "Reset" and resp == "Ok"

    def encode_inv(self, inv, accounts):
        if inv not in self.INV:
            raise EncodeError(f"unknown TicketDispenser request {inv!r}")
        return self.INV[inv], 0, 0, 0

    def encode_resp(self, resp):
        if resp == "Ok":
            return 1, 0
        if isinstance(resp, tuple) and len(resp) == 2 and resp[0] == "Number":
            return 0, _i32(resp[1])
        raise EncodeError(f"unknown TicketDispenser response {resp!r}")

    def decode_inv(self, code, a, b, val, accounts):
        return self.INV_NAMES[code]

    def decode_resp(self, code, val):
        return ("Number", val) if code == 0 else "Ok"

    def pack_model0(self, model0, accounts):
        if model0 is None:
            return None
        return TicketModel(1, 0, _i32(model0))

    def show_model(self, m):
        return "Nothing" if m is None else f"Just {m}"

    def show_inv(self, inv):
        return inv

    def show_resp(self, resp):
        return "Ok" if resp == "Ok" else f"Number {resp[1]}"


# ---------------------------------------------------------------------------
# Bank
# ---------------------------------------------------------------------------

class BankModel(ctypes.Structure):
    _fields_ = [("exists", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("balance", ctypes.c_int64 * BANK_MAX_ACCOUNTS)]


BANK_REQ = {"OpenAccount": 0, "Deposit": 1, "Withdraw": 2, "CheckBalance": 3, "Transfer": 4}
BANK_REQ_NAMES = {v: k for k, v in BANK_REQ.items()}
BANK_RESP = {"AccountCreated": 0, "DepositMade": 1, "WithdrawalMade": 2, "TransferMade": 3,
             "AccountAlreadyExists": 4, "AccountDoesntExist": 5, "InsufficientFunds": 6}
BANK_RESP_NAMES = {v: k for k, v in BANK_RESP.items()}
BANK_BALANCE = 7


def _bank_deposit(model, a, money):
    m2 = dict(model)
    m2[a] = model[a] + money if a in model else money
    return m2


def _bank_withdraw(model, a, money):
    m2 = dict(model)
    m2[a] = model[a] - money if a in model else money
    return m2


class Bank(DeviceModel):
    name = "bank"
    model_id = MODEL_BANK

    @property
    def init_model(self):                           # M.empty
        return {}

    @staticmethod
    def transition(model, ev):                      # Bank.hs:92-101  (next')
        kind, x = ev
        if kind == "R":
            return model
        op = x[0]
        if op == "OpenAccount":
            if x[1] in model:
                return model
            m2 = dict(model)
            m2[x[1]] = 0
            return m2
        if op == "Deposit":
            return _bank_deposit(model, x[1], x[2])
        if op == "Withdraw":
            return _bank_withdraw(model, x[1], x[2])
        if op == "CheckBalance":
            return model
        if op == "Transfer":
            return _bank_deposit(_bank_withdraw(model, x[1], x[2]), x[3], x[2])
        raise ValueError(x)

    @staticmethod
    def postcondition(model, req, resp):            # Bank.hs:118-131  (post)
        if not all(v >= 0 for v in model.values()):     # invariant, :103-104
            return False
        op = req[0]
        if op == "OpenAccount":
            return resp == ("AccountAlreadyExists" if req[1] in model else "AccountCreated")
        if op == "Deposit":
            return resp == "DepositMade"
        if op in ("Withdraw", "Transfer"):
            ok = req[1] in model and model[req[1]] >= req[2]
            made = "WithdrawalMade" if op == "Withdraw" else "TransferMade"
            return resp == (made if ok else "InsufficientFunds")
        if op == "CheckBalance":
            if isinstance(resp, tuple) and resp[0] == "Balance":
                if req[1] not in model:
                    raise ModelError("Map.!: given key is not an element in the map")
                return resp[1] == model[req[1]]
            return False
        raise ValueError(req)

    # accounts are arbitrary Eq/Ord values (ProcessIds in the reference);
    # each history maps them to dense indices 0..7 in order of first mention,
    # after the keys of a non-empty model0.
    def new_account_map(self, model0):
        accounts = {}
        for k in (model0 or {}):
            accounts[k] = len(accounts)
        return accounts

    @staticmethod
    def _acc(accounts, a):
        if a not in accounts:
            if len(accounts) >= BANK_MAX_ACCOUNTS:
                raise EncodeError("more than 8 accounts in one history")
            accounts[a] = len(accounts)
        return accounts[a]

    def encode_inv(self, req, accounts):
        if not isinstance(req, tuple) or not req or req[0] not in BANK_REQ:
            raise EncodeError(f"unknown Bank request {req!r}")
        op = req[0]
        code = BANK_REQ[op]
        if op in ("OpenAccount", "CheckBalance"):
            if len(req) != 2:
                raise EncodeError(repr(req))
            return code, self._acc(accounts, req[1]), 0, 0
        if op in ("Deposit", "Withdraw"):
            if len(req) != 3:
                raise EncodeError(repr(req))
            return code, self._acc(accounts, req[1]), 0, _i32(req[2])
        if len(req) != 4:
            raise EncodeError(repr(req))
        a = self._acc(accounts, req[1])
        b = self._acc(accounts, req[3])
        return code, a, b, _i32(req[2])

    def encode_resp(self, resp):
        if isinstance(resp, tuple) and len(resp) == 2 and resp[0] == "Balance":
            return BANK_BALANCE, _i32(resp[1])
        if isinstance(resp, str) and resp in BANK_RESP:
            return BANK_RESP[resp], 0
        raise EncodeError(f"unknown Bank response {resp!r}")

    def decode_inv(self, code, a, b, val, accounts):
        inv_acc = {v: k for k, v in accounts.items()}
        op = BANK_REQ_NAMES[code]
        if op in ("OpenAccount", "CheckBalance"):
            return (op, inv_acc[a])
        if op in ("Deposit", "Withdraw"):
            return (op, inv_acc[a], val)
        return (op, inv_acc[a], val, inv_acc[b])

    def decode_resp(self, code, val):
        return ("Balance", val) if code == BANK_BALANCE else BANK_RESP_NAMES[code]

    def pack_model0(self, model0, accounts):
        if not model0:
            return None
        m = BankModel()
        for k, v in model0.items():
            idx = accounts[k]
            m.exists |= 1 << idx
            m.balance[idx] = _i32(v)
        return m

    def show_model(self, model):
        items = ",".join(f"({k!r},{v})" for k, v in sorted(model.items(), key=lambda kv: repr(kv[0])))
        return f"fromList [{items}]"

    def show_inv(self, req):
        return " ".join(str(x) for x in req)

    def show_resp(self, resp):
        return resp if isinstance(resp, str) else f"Balance {resp[1]}"


TICKET = TicketDispenser()
BANK = Bank()

BY_ID = {MODEL_TICKET: TICKET, MODEL_BANK: BANK}
BY_NAME = {"ticket": TICKET, "bank": BANK}
