{-# LANGUAGE FlexibleInstances     #-}
{-# LANGUAGE MultiParamTypeClasses #-}
{-# OPTIONS_GHC -Wno-orphans #-}

-- | 'DeviceModel' instances for the reference's two models: the device
-- functors QSMD_MODEL_BANK (test/Bank.hs:41-131) and QSMD_MODEL_TICKET
-- (test/TicketDispenser.hs:51-102).  The constructor codes are
-- include/qsmd.h's (QSMD_BANK_* / QSMD_TICKET_*), which follow the Haskell
-- declaration order.
module DeviceInstances () where

import           Control.Distributed.Process
                   (ProcessId)
import qualified Data.Map               as M

import qualified Bank
import           Linearisability.Device
import qualified TicketDispenser        as TD

-- Bank: the model is @ModelF ProcessId = Map ProcessId Integer@ and the
-- accounts are the ProcessIds the requests name (test/Bank.hs:41-60).
instance DeviceModel (M.Map ProcessId Integer) Bank.BankRequest Bank.BankResponse ProcessId where
  deviceModelId _ = qsmdModelBank
  encodeInv _ req = Just $ case req of
    Bank.OpenAccount a      -> Invocation 0 [a] 0
    Bank.Deposit a money    -> Invocation 1 [a] money
    Bank.Withdraw a money   -> Invocation 2 [a] money
    Bank.CheckBalance a     -> Invocation 3 [a] 0
    Bank.Transfer a money b -> Invocation 4 [a, b] money
  encodeResp _ resp = Just $ case resp of
    Bank.AccountCreated       -> (0, 0)
    Bank.DepositMade          -> (1, 0)
    Bank.WithdrawalMade       -> (2, 0)
    Bank.TransferMade         -> (3, 0)
    Bank.AccountAlreadyExists -> (4, 0)
    Bank.AccountDoesntExist   -> (5, 0)
    Bank.InsufficientFunds    -> (6, 0)
    Bank.Balance money        -> (7, money)
  deviceModel0 m = BankModel0 (M.toList m)

-- TicketDispenser: the model is @Maybe Int@; no accounts.
instance DeviceModel (Maybe Int) TD.Request TD.Response () where
  deviceModelId _ = qsmdModelTicket
  encodeInv _ TD.TakeTicket = Just (Invocation 0 [] 0)
  encodeInv _ TD.Reset      = Just (Invocation 1 [] 0)
  encodeResp _ (TD.Number i) = Just (0, toInteger i)
  encodeResp _ TD.Ok         = Just (1, 0)
  deviceModel0 m = TicketModel0 m
