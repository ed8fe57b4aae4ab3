"""qsmd -- MI355X-native drop-in for ``linearisable`` of
advancedtelematic/quickcheck-state-machine-distributed (src/Linearisability.hs).

Host-side mirror of the reference interface; the search runs in hand-written
HIP kernels (csrc/*.hip, lib/libqsmd.so) behind the C ABI of include/qsmd.h.
"""

from .codec import Left, Right, encode, decode_history, STATUS_NAMES  # noqa: F401
from .models import BANK, TICKET, Bank, TicketDispenser, DeviceModel, ModelError, EncodeError  # noqa: F401
from .linearisability import (linearisable, linearisable_batch, trace, wellformed,  # noqa: F401
                              replay_witness, CheckResult, NotSequential, BudgetExceeded)
from . import device, gen  # noqa: F401
