{-# LANGUAGE FlexibleContexts         #-}
{-# LANGUAGE ForeignFunctionInterface #-}
{-# LANGUAGE FunctionalDependencies   #-}
{-# LANGUAGE MultiParamTypeClasses    #-}
{-# LANGUAGE ScopedTypeVariables      #-}

-- | GPU drop-in for 'Linearisability.linearisable'
-- (src/Linearisability.hs:52-69 of advancedtelematic/quickcheck-state-machine-distributed).
--
-- 'linearisableDevice' keeps the reference's signature and argument order:
--
-- > linearisable       :: Eq pid => (model -> Either inv resp -> model)
-- >                     -> (model -> inv -> resp -> Bool) -> model -> History pid inv resp -> Bool
-- > linearisableDevice :: (Eq pid, DeviceModel model inv resp acc)
-- >                     => (model -> Either inv resp -> model)
-- >                     -> (model -> inv -> resp -> Bool) -> model -> History pid inv resp -> Bool
--
-- The search runs on the GPU in libqsmd.so (include/qsmd.h) with the model's
-- device functor (selected by 'deviceModelId'); the closures passed here
-- replay the witness the device returns, so every True is re-checked on the
-- host against the Haskell model.  A model exception on the device (Bank's
-- @Map.!@, test/Bank.hs:128) is raised as the reference raises it.
--
-- Link with @extra-libraries: qsmd@ and @extra-lib-dirs:@ pointing at
-- quickcheck-state-machine-distributed_amd/lib.  This module is source only:
-- no GHC exists in the image it was written in (INTEGRATION.md §1).
module Linearisability.Device
  ( -- * Models the device knows
    DeviceModel(..)
  , Invocation(..)
  , Model0(..)
    -- * The reference's function, on the GPU
  , linearisableDevice
  , linearisableDeviceIO
  , linearisableBatch
  , Verdict(..)
  , DeviceError(..)
    -- * Encoding (exposed for tests)
  , EncodedEvent(..)
  , encodeHistory
  , qsmdModelTicket
  , qsmdModelBank
  ) where

import           Control.Concurrent.MVar
                   (MVar, modifyMVar, newMVar)
import           Control.Exception
                   (ErrorCall(..), Exception, throw, throwIO)
import           Control.Monad
                   (forM_, unless, when)
import           Data.Bits
                   (shiftL, (.|.))
import           Data.Int
                   (Int32, Int64)
import           Data.List
                   (elemIndex)
import qualified Data.Map.Strict         as M
import           Data.Word
                   (Word16, Word32, Word64, Word8)
import           Foreign.C.String
                   (CString, peekCString)
import           Foreign.C.Types
                   (CInt(..))
import           Foreign.Marshal.Alloc
                   (alloca, allocaBytes)
import           Foreign.Marshal.Array
                   (peekArray)
import           Foreign.Ptr
                   (Ptr, castPtr, nullPtr, plusPtr)
import           Foreign.Storable
                   (peek, pokeByteOff)
import           System.IO.Unsafe
                   (unsafePerformIO)

import           Linearisability
                   (History)

------------------------------------------------------------------------
-- The C ABI (include/qsmd.h)

data QsmdCtx

foreign import ccall safe "qsmd_open"
  c_open :: Ptr (Ptr QsmdCtx) -> CInt -> IO CInt
foreign import ccall safe "qsmd_last_error"
  c_last_error :: Ptr QsmdCtx -> IO CString
foreign import ccall safe "qsmd_timed_out"
  c_timed_out :: Ptr QsmdCtx -> Ptr CInt -> IO CInt
-- `safe`: a call can run for a long time and must not block the other
-- capabilities of the -threaded RTS (package.yaml:48-51).
foreign import ccall safe "qsmd_check_batch"
  c_check_batch
    :: Ptr QsmdCtx -> Word32
    -> Ptr () -> Word64            -- qsmd_hdr[n_hist]          (16 B each)
    -> Ptr () -> Word64            -- qsmd_event[n_events]      (8 B each)
    -> Ptr () -> Word32 -> Word64  -- model0 (NULL = initModel), flags, max_nodes
    -> Ptr Word8 -> Ptr Word64 -> Ptr Word8 -> Ptr ()   -- status, nodes, witness, totals
    -> IO CInt

qsmdModelTicket, qsmdModelBank :: Word32
qsmdModelTicket = 1
qsmdModelBank   = 2

flagExhaustive, flagWitness :: Word32
flagExhaustive = 1
flagWitness    = 4

witnessEnd :: Word8
witnessEnd = 0xFF

------------------------------------------------------------------------
-- Models

-- | An invocation as the device sees it: the request's constructor code
-- (include/qsmd.h QSMD_BANK_* / QSMD_TICKET_*), the accounts it names (Bank:
-- @a@, then @b@ for Transfer) and its value.
data Invocation acc = Invocation
  { invCode     :: !Word8
  , invAccounts :: [acc]
  , invValue    :: !Integer
  }

-- | The initial model, as the device takes it (qsmd_ticket_model /
-- qsmd_bank_model).
data Model0 acc
  = TicketModel0 (Maybe Int)
  | BankModel0 [(acc, Integer)]    -- the keys and values of the initial Map

-- | The link between a model's closures and a device functor.  @acc@ is the
-- type the model keys its state by (Bank: the account 'ProcessId';
-- TicketDispenser: '()').  Instances for the reference's two models are in
-- hs/DeviceInstances.hs.
class Ord acc => DeviceModel model inv resp acc | model -> inv resp acc where
  deviceModelId :: model -> Word32
  encodeInv     :: model -> inv -> Maybe (Invocation acc)   -- Nothing: no device code
  encodeResp    :: model -> resp -> Maybe (Word8, Integer)  -- (constructor code, value)
  deviceModel0  :: model -> Model0 acc

-- | One call's answer per history.
data Verdict
  = Linearisable [Int]      -- ^ the witness: invocation event indices, in order
  | NotLinearisable
  | ModelError              -- ^ the reference raises (Map.!)
  | NotEncodable String     -- ^ outside include/qsmd.h's encoding (INTEGRATION.md §3)
  deriving (Eq, Show)

newtype DeviceError = DeviceError String
  deriving Show

instance Exception DeviceError

------------------------------------------------------------------------
-- Encoding (include/qsmd.h layout)

-- | One qsmd_event: kind << 7 | dense pid, constructor code, accounts a and b, value.
data EncodedEvent = EncodedEvent !Word8 !Word8 !Word8 !Word8 !Int32
  deriving (Eq, Show)

inInt32 :: Integer -> Maybe Int32
inInt32 v
  | v >= toInteger (minBound :: Int32) && v <= toInteger (maxBound :: Int32) = Just (fromInteger v)
  | otherwise = Nothing

-- | Dense pids in order of first use (the reference compares pids with Eq
-- only, src/Linearisability.hs:30-45); dense accounts after model0's keys,
-- in order of first mention.  Returns (n_pid, events) or why it cannot.
encodeHistory
  :: forall model inv resp acc pid. (Eq pid, DeviceModel model inv resp acc)
  => model -> History pid inv resp -> Either String (Int, [EncodedEvent])
encodeHistory m hist
  | length hist > 128 = Left "more than 128 events"
  | otherwise = go [] accounts0 hist []
  where
    accounts0 :: M.Map acc Word8
    accounts0 = case deviceModel0 m of
      BankModel0 kvs -> M.fromList (zip (map fst kvs) [0 ..])
      TicketModel0 _ -> M.empty

    go pids _ [] acc = Right (length pids, reverse acc)
    go pids accts ((pid, ev) : rest) acc = do
      let (p, pids') = case elemIndex pid pids of
            Just i  -> (i, pids)
            Nothing -> (length pids, pids ++ [pid])
      when (p >= 128) (Left "more than 128 pids")
      case ev of
        Left inv -> case encodeInv m inv of
          Nothing -> Left "no device code for an invocation"
          Just (Invocation code accs val) -> do
            (idxs, accts') <- number accts accs
            v <- maybe (Left "value outside Int32") Right (inInt32 val)
            let (a, b) = case idxs of
                  [x]    -> (x, 0)
                  [x, y] -> (x, y)
                  _      -> (0, 0)
            go pids' accts' rest (EncodedEvent (fromIntegral p) code a b v : acc)
        Right resp -> case encodeResp m resp of
          Nothing -> Left "no device code for a response"
          Just (code, val) -> do
            v <- maybe (Left "value outside Int32") Right (inInt32 val)
            go pids' accts rest (EncodedEvent (0x80 .|. fromIntegral p) code 0 0 v : acc)

    number accts [] = Right ([], accts)
    number accts (x : xs) = do
      (i, accts1) <- case M.lookup x accts of
        Just i  -> Right (i, accts)
        Nothing
          | M.size accts >= 8 -> Left "more than 8 Bank accounts in one history"
          | otherwise         -> Right (fromIntegral (M.size accts), M.insert x (fromIntegral (M.size accts)) accts)
      (is, accts2) <- number accts1 xs
      Right (i : is, accts2)

------------------------------------------------------------------------
-- The device context: one per process (one process per GPU), opened on
-- first use.

{-# NOINLINE globalCtx #-}
globalCtx :: MVar (Maybe (Ptr QsmdCtx))
globalCtx = unsafePerformIO (newMVar Nothing)

withCtx :: (Ptr QsmdCtx -> IO a) -> IO a
withCtx k = modifyMVar globalCtx $ \mctx -> do
  ctx <- case mctx of
    Just c  -> return c
    Nothing -> alloca $ \pp -> do
      rc <- c_open pp 0
      unless (rc == 0) (throwIO (DeviceError ("qsmd_open failed: " ++ show rc)))
      peek pp
  r <- k ctx
  return (Just ctx, r)

------------------------------------------------------------------------
-- Checking

-- | Check histories of one model in one device call (the throughput path).
-- The first argument is model0 (the reference's @initModel@ or any other).
linearisableBatch
  :: forall model inv resp acc pid. (Eq pid, DeviceModel model inv resp acc)
  => model -> [History pid inv resp] -> IO [Verdict]
linearisableBatch m hists =
  withCtx $ \ctx ->
    allocaBytes (max 16 (16 * nHist)) $ \hdr ->
    allocaBytes (max 8 (8 * nEv)) $ \evp ->
    allocaBytes (max 1 nEv) $ \wit ->
    allocaBytes (max 1 nHist) $ \st ->
    allocaBytes 80 $ \m0buf -> do
      forM_ (zip3 [0 :: Int ..] enc offs) (pokeHeader hdr)
      forM_ (zip [0 :: Int ..] (concat ok)) (pokeEvent evp)
      mm0 <- pokeModel0 (deviceModel0 m) m0buf
      case mm0 of
        Nothing  -> return (map (const (NotEncodable "model0 outside the device encoding")) hists)
        Just m0p -> do
          rc <- c_check_batch ctx (deviceModelId m) (castPtr hdr) (fromIntegral nHist)
                              (castPtr evp) (fromIntegral nEv) m0p (flagExhaustive .|. flagWitness) 0
                              st nullPtr wit nullPtr
          unless (rc == 0) $ do
            msg <- c_last_error ctx >>= peekCString
            throwIO (DeviceError ("qsmd_check_batch failed (" ++ show rc ++ "): " ++ msg))
          status <- peekArray nHist st
          ws     <- peekArray nEv wit
          -- max_nodes is 0 here: a BUDGET status can only come from the
          -- safety net (qsmd_set_time_limit_ms); say so rather than guess
          when (4 `elem` status) $ alloca $ \tp -> do
            _ <- c_timed_out ctx tp
            timed <- peek tp
            throwIO (DeviceError (if timed /= 0
                                    then "the device time limit fired before every verdict was decided"
                                    else "unexpected BUDGET status without a node limit"))
          return (zipWith3 (verdict ws) enc offs status)
  where
    enc   = map (encodeHistory m) hists
    ok    = [ evs | Right (_, evs) <- enc ]
    nHist = length hists
    nEv   = sum (map length ok)
    offs  = scanl (+) 0 [ either (const 0) (length . snd) e | e <- enc ]

    -- qsmd_hdr: {ev_off u32, n_ev u16, n_pid u8, model_id u8, tag u32, 0 u32}
    pokeHeader :: Ptr () -> (Int, Either String (Int, [EncodedEvent]), Int) -> IO ()
    pokeHeader hdr (i, e, off) = do
      let base = hdr `plusPtr` (16 * i)
      pokeByteOff base 0 (fromIntegral off :: Word32)
      case e of
        Right (nPid, evs) -> do
          pokeByteOff base 4 (fromIntegral (length evs) :: Word16)
          pokeByteOff base 6 (fromIntegral nPid :: Word8)
          pokeByteOff base 7 (fromIntegral (deviceModelId m) :: Word8)
        Left _ -> do                            -- model_id 0xFF: QSMD_STATUS_ENCODE_ERROR
          pokeByteOff base 4 (0 :: Word16)
          pokeByteOff base 6 (0 :: Word8)
          pokeByteOff base 7 (0xFF :: Word8)
      pokeByteOff base 8 (fromIntegral i :: Word32)
      pokeByteOff base 12 (0 :: Word32)

    -- qsmd_event: {kind << 7 | pid u8, code u8, a u8, b u8, val i32}
    pokeEvent :: Ptr () -> (Int, EncodedEvent) -> IO ()
    pokeEvent evp (j, EncodedEvent kp code a b v) = do
      let base = evp `plusPtr` (8 * j)
      pokeByteOff base 0 kp
      pokeByteOff base 1 code
      pokeByteOff base 2 a
      pokeByteOff base 3 b
      pokeByteOff base 4 v

    verdict :: [Word8] -> Either String (Int, [EncodedEvent]) -> Int -> Word8 -> Verdict
    verdict _ (Left why) _ _ = NotEncodable why
    verdict ws (Right (_, evs)) off s = case s of
      1 -> Linearisable [ fromIntegral w | w <- takeWhile (/= witnessEnd) (take (length evs) (drop off ws)) ]
      0 -> NotLinearisable
      2 -> ModelError
      3 -> NotEncodable "rejected by the device encoding"
      c -> throw (DeviceError ("unexpected status " ++ show c))

    -- Nothing: model0 outside the device's encoding (> 8 accounts, a value
    -- beyond Int32); Just nullPtr: the reference's initModel
    pokeModel0 :: Model0 acc -> Ptr () -> IO (Maybe (Ptr ()))
    pokeModel0 (TicketModel0 Nothing) _ = return (Just nullPtr)
    pokeModel0 (TicketModel0 (Just n)) p = case inInt32 (toInteger n) of
      Nothing -> return Nothing
      Just v  -> do
        pokeByteOff p 0 (1 :: Word32)
        pokeByteOff p 4 (0 :: Word32)
        pokeByteOff p 8 (fromIntegral v :: Int64)
        return (Just p)
    pokeModel0 (BankModel0 []) _ = return (Just nullPtr)
    pokeModel0 (BankModel0 kvs) p
      | length kvs > 8 = return Nothing
      | otherwise = case mapM (inInt32 . snd) kvs of
          Nothing -> return Nothing
          Just vs -> do
            let exists = foldr (.|.) 0 [ (1 :: Word32) `shiftL` i | i <- [0 .. length kvs - 1] ]
            pokeByteOff p 0 exists
            pokeByteOff p 4 (0 :: Word32)
            forM_ [0 .. 7 :: Int] $ \i -> pokeByteOff p (8 + 8 * i) (0 :: Int64)
            forM_ (zip [0 :: Int ..] vs) $ \(i, v) -> pokeByteOff p (8 + 8 * i) (fromIntegral v :: Int64)
            return (Just p)

-- | 'linearisable' with the reference's argument order, on the device; the
-- closures replay the witness of every True on the host.
linearisableDeviceIO
  :: (Eq pid, DeviceModel model inv resp acc)
  => (model -> Either inv resp -> model)
  -> (model -> inv -> resp -> Bool)
  -> model
  -> History pid inv resp
  -> IO Bool
linearisableDeviceIO transition postcondition model0 hist = do
  vs <- linearisableBatch model0 [hist]
  case vs of
    [Linearisable w]
      | replay transition postcondition model0 hist w -> return True
      | otherwise -> throwIO (DeviceError "the device's witness does not replay on the host model")
    [NotLinearisable]  -> return False
    [ModelError]       -> throwIO (ErrorCall "Map.!: given key is not an element in the map")
    [NotEncodable why] -> throwIO (DeviceError ("history outside the device encoding: " ++ why))
    _                  -> throwIO (DeviceError "one verdict expected")

-- | The pure drop-in: @linearisable@ -> @linearisableDevice@ at a call site
-- (test/Bank.hs:285, test/TicketDispenser.hs:253, :320).
{-# NOINLINE linearisableDevice #-}
linearisableDevice
  :: (Eq pid, DeviceModel model inv resp acc)
  => (model -> Either inv resp -> model)
  -> (model -> inv -> resp -> Bool)
  -> model
  -> History pid inv resp
  -> Bool
linearisableDevice transition postcondition model0 hist =
  unsafePerformIO (linearisableDeviceIO transition postcondition model0 hist)

-- | Replay a witness (SURVEY.md §8a Lemma L1) as a path of the reference's
-- tree: each chosen invocation j must be a root of
-- @interleavings rest@ -- a remaining invocation inside the
-- 'takeInvocations' prefix (before the first remaining response,
-- src/Linearisability.hs:25-28) whose pid has a remaining response
-- (findResponse, :30-34); the operation is (its pid p, its inv, the first
-- remaining response of p); the first remaining invocation and response of p
-- are removed (filter1, :41,:47-50).  The path must end at a leaf (no root
-- left: @any' [] = True@, :67), and the empty witness stands only for the
-- empty history (@linearisable _ _ _ [] = True@, :59; a non-empty history
-- with no root is False, :60).  A truncated witness, or one that starts an
-- operation after a pending response, is rejected.
replay
  :: Eq pid
  => (model -> Either inv resp -> model)
  -> (model -> inv -> resp -> Bool)
  -> model -> History pid inv resp -> [Int] -> Bool
replay _ _ _ hist [] = null hist
replay transition postcondition model0 hist ws0 = go model0 (zip [0 ..] hist) ws0
  where
    go _ rest [] = null (roots rest)
    go m rest (j : js) = case lookup j (prefix rest) of
      Just (pid, Left inv) -> case firstResp pid rest of
        Just (k, resp) ->
          postcondition m inv resp
            && go (transition (transition m (Left inv)) (Right resp))
                  (dropFirstInv pid (filter ((/= k) . fst) rest)) js
        Nothing -> False
      _ -> False
    -- takeInvocations: the remaining events before the first remaining response
    prefix = takeWhile (isInv . snd)
    -- the roots of interleavings rest: prefix invocations whose pid has a response
    roots rest = [ i | (i, (pid, Left _)) <- prefix rest, Just _ <- [firstResp pid rest] ]
    firstResp pid rest = case [ (k, r) | (k, (q, Right r)) <- rest, q == pid ] of
      kr : _ -> Just kr
      []     -> Nothing
    isInv (_, Left _) = True
    isInv _           = False
    dropFirstInv pid evs = case break isInvOf evs of
      (before, _ : after) -> before ++ after
      (before, [])        -> before
      where
        isInvOf (_, (q, Left _)) = q == pid
        isInvOf _                = False
