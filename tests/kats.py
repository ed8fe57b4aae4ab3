"""Known-answer histories.  KAT-2 is the reference's own
example output, test/TicketDispenser.hs:326-347 (shrunk program
([Reset],[TakeTicket,TakeTicket]); the history's verdict is "Can't
linearise"); the others are hand-derived from src/Linearisability.hs:25-69."""

L = lambda x: ("L", x)  # noqa: E731
R = lambda x: ("R", x)  # noqa: E731

KATS = {
    # name: (model, history, expected status, expected nodes)
    "KAT1_empty": ("ticket", [], "lin", 0),
    "KAT2_reference_example": ("ticket", [
        ("8", L("Reset")), ("8", R("Ok")), ("8", L("TakeTicket")), ("8", L("TakeTicket")),
        ("8", R(("Number", 2))), ("8", R(("Number", 1)))], "nonlin", 3),
    "KAT3_distinct_pids": ("ticket", [
        ("c1", L("Reset")), ("c1", R("Ok")), ("c1", L("TakeTicket")), ("c2", L("TakeTicket")),
        ("c2", R(("Number", 2))), ("c1", R(("Number", 1)))], "lin", 3),
    "KAT4_lone_invocation": ("ticket", [("p", L("TakeTicket"))], "nonlin", 0),
    "KAT5_pending_is_leaf": ("ticket", [
        ("p", L("Reset")), ("p", R("Ok")), ("q", L("TakeTicket"))], "lin", 1),
    "KAT6_response_first": ("ticket", [("p", R("Ok")), ("p", L("Reset"))], "nonlin", 0),
    "KAT7_bank_concurrent": ("bank", [
        ("a", L(("OpenAccount", "a"))), ("a", R("AccountCreated")),
        ("b", L(("OpenAccount", "b"))), ("b", R("AccountCreated")),
        ("b", L(("Deposit", "b", 10))), ("b", R("DepositMade")),
        ("a", L(("CheckBalance", "a"))), ("b", L(("Transfer", "b", 5, "a"))),
        ("a", R(("Balance", 3))), ("b", R("TransferMade"))], "nonlin", 6),
    # Map.! on a missing account (test/Bank.hs:128) -> the reference raises
    "KAT8_bank_map_error": ("bank", [
        ("a", L(("CheckBalance", "a"))), ("a", R(("Balance", 0)))], "error", 1),
    # the same request answered by a non-Balance constructor does not force Map.!
    "KAT9_bank_no_error": ("bank", [
        ("a", L(("CheckBalance", "a"))), ("a", R("AccountDoesntExist"))], "nonlin", 1),
    # Bank KATs 10-16, hand-derived from test/Bank.hs:92-131 (next', invariant,
    # post) and src/Linearisability.hs:52-69; each pins one clause:
    # Withdraw on an absent account inserts +m (insertWith keeps the new value)
    "KAT10_bank_withdraw_creates": ("bank", [
        ("a", L(("Withdraw", "a", 5))), ("a", R("InsufficientFunds")),
        ("a", L(("CheckBalance", "a"))), ("a", R(("Balance", 5)))], "lin", 2),
    # next' ignores the response (the refused Withdraw still subtracts), and
    # the invariant is checked on the pre-state of the next step
    "KAT11_bank_invariant_prestate": ("bank", [
        ("a", L(("OpenAccount", "a"))), ("a", R("AccountCreated")),
        ("a", L(("Withdraw", "a", 5))), ("a", R("InsufficientFunds")),
        ("a", L(("Deposit", "a", 1))), ("a", R("DepositMade"))], "nonlin", 3),
    # Transfer = Withdraw then Deposit, on one account: absent -> +7 -> 14
    "KAT12_bank_self_transfer": ("bank", [
        ("a", L(("Transfer", "a", 7, "a"))), ("a", R("InsufficientFunds")),
        ("a", L(("CheckBalance", "a"))), ("a", R(("Balance", 14)))], "lin", 2),
    # OpenAccount on an existing account: AlreadyExists, balance kept
    "KAT13_bank_open_existing": ("bank", [
        ("a", L(("Deposit", "a", 3))), ("a", R("DepositMade")),
        ("a", L(("OpenAccount", "a"))), ("a", R("AccountAlreadyExists")),
        ("a", L(("CheckBalance", "a"))), ("a", R(("Balance", 3)))], "lin", 3),
    # two concurrent operations, both orders tried and both fail: Deposit
    # first expects WithdrawalMade; Withdraw first is refused, leaves -4, and
    # the Deposit after it meets the broken invariant
    "KAT14_bank_both_orders_fail": ("bank", [
        ("a", L(("OpenAccount", "a"))), ("a", R("AccountCreated")),
        ("a", L(("Deposit", "a", 10))), ("b", L(("Withdraw", "a", 4))),
        ("a", R("DepositMade")), ("b", R("InsufficientFunds"))], "nonlin", 5),
    # Map.! after a successful prefix: the error ends the search at node 2
    "KAT15_bank_error_after_prefix": ("bank", [
        ("a", L(("OpenAccount", "a"))), ("a", R("AccountCreated")),
        ("b", L(("CheckBalance", "b"))), ("b", R(("Balance", 0)))], "error", 2),
    # Nothing < Just m: a Transfer from an absent account must be refused
    "KAT16_bank_nothing_below_just": ("bank", [
        ("a", L(("Transfer", "a", 5, "b"))), ("a", R("TransferMade"))], "nonlin", 1),
}

# The trace text of the reference's example (test/TicketDispenser.hs:329-344),
# pid shown as the suffix after the last ':' (prettyPrintProcessId, :73-74).
KAT2_TRACE = (
    "Nothing\n  ==> Reset  [8]\n"
    "Just 0\n  <== Ok  [8]\n"
    "Just 0\n  ==> TakeTicket  [8]\n"
    "Just 1\n  ==> TakeTicket  [8]\n"
    "Just 2\n  <== Number 2  [8]\n"
    "Just 2\n  <== Number 1  [8]\n")
