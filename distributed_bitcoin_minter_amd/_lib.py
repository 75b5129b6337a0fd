"""ctypes binding of libbtcminer.so (C ABI: include/btcminer.h).

The library is built in-tree (``make -C distributed_bitcoin_minter_amd/csrc``)
and loaded from this package directory.  There is no fallback: if the
library is missing, or there is no gfx950 device, calls raise.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# BTCMINER_LIB overrides the library path (used to A/B kernel build variants;
# they must be built from the same ABI version)
LIB_PATH = os.environ.get("BTCMINER_LIB") or os.path.join(_HERE, "libbtcminer.so")

BM_OK = 0
BM_EINVAL = -1
BM_ENODEV = -2
BM_EHIP = -3
BM_ERCCL = -4
BM_ENOMEM = -5
BM_EINTERNAL = -6
BM_EPEER = -7
BM_ETIMEDOUT = -8
BM_MAX_LAUNCH_STATS = 64
BM_MAX_STAT_DEVICES = 16
BM_RCCL_ID_BYTES = 128
BM_ABI_VERSION = 7
BM_DEFAULT_PEER_TIMEOUT_MS = 600_000
BM_COMBINE_AUTO, BM_COMBINE_RCCL, BM_COMBINE_HOST = 0, 1, 2
# bm_stats_t.combine_used
BM_COMBINED_NONE, BM_COMBINED_RCCL, BM_COMBINED_HOST, BM_COMBINED_LOCAL = 0, 1, 2, 3
COMBINED_NAMES = {0: "none", 1: "rccl", 2: "host", 3: "local"}
U64_MAX = (1 << 64) - 1

c_u64 = ctypes.c_uint64
c_u32 = ctypes.c_uint32
c_i32 = ctypes.c_int32


class Result(ctypes.Structure):
    _fields_ = [("hash", c_u64), ("nonce", c_u64)]


class LaunchStat(ctypes.Structure):
    _fields_ = [("device", c_i32), ("p", c_i32), ("nbv", c_i32), ("pad_block", c_i32), ("digits", c_i32),
                ("inner_digits", c_i32), ("nonces", c_u64), ("grid", c_u32), ("tasks_per_thread", c_u32),
                ("ms", ctypes.c_double), ("clock_ghz", ctypes.c_double)]


class Stats(ctypes.Structure):
    _fields_ = [("launches", c_u32), ("recorded", c_u32), ("wall_ms", ctypes.c_double),
                ("kernel_ms", ctypes.c_double), ("span_ms", ctypes.c_double), ("nonces", c_u64),
                ("combine_used", c_i32), ("rccl_status", c_i32), ("devices", c_u32), ("reserved", c_u32),
                ("dev_nonces", c_u64 * BM_MAX_STAT_DEVICES), ("dev_span_ms", ctypes.c_double * BM_MAX_STAT_DEVICES),
                ("rccl_nranks", c_i32), ("rccl_rank", c_i32), ("dev_rccl_rank", c_i32 * BM_MAX_STAT_DEVICES),
                ("dev_rccl_device", c_i32 * BM_MAX_STAT_DEVICES),
                # ABI 7: the RCCL version, the communicator's set-up time, the allgather's
                # event pair and each device's start against the earliest device's
                ("rccl_version", c_i32), ("start_threads", c_i32), ("rccl_init_ms", ctypes.c_double),
                ("rccl_allgather_ms", ctypes.c_double), ("combine_ms", ctypes.c_double),
                ("dev_allgather_ms", ctypes.c_double * BM_MAX_STAT_DEVICES),
                ("dev_start_ms", ctypes.c_double * BM_MAX_STAT_DEVICES),
                ("launch", LaunchStat * BM_MAX_LAUNCH_STATS)]


class Segment(ctypes.Structure):
    _fields_ = [("p", c_i32), ("nbv", c_i32), ("pad_block", c_i32), ("digits", c_i32), ("nd", c_i32),
                ("max_inner", c_i32), ("vlo", c_u64), ("vhi", c_u64), ("nonce_base", c_u64),
                ("mid", c_u32 * 8), ("tmpl", c_u32 * 32), ("pad_w", c_u32 * 16)]


class BtcMinerError(RuntimeError):
    def __init__(self, status, what):
        self.status = status
        super().__init__(f"{what}: {strerror(status)} ({status})")


_lib = None
_variants = {}
# The same library built with BM_CLOCK_PROBE=1 (`make -C csrc probe`): its
# launches stamp the shader clock.  bench.py loads it beside the product
# library, only to measure the clock under the dominant kernel after the
# timed region; nothing else uses it.
PROBE_LIB_PATH = os.path.join(_HERE, "libbtcminer_probe.so")


def load(path=None):
    """Load libbtcminer.so once (or, with a path, another build of the same
    ABI, e.g. PROBE_LIB_PATH); raises OSError if it has not been built."""
    global _lib
    if path is not None and os.path.abspath(path) != os.path.abspath(LIB_PATH):
        path = os.path.abspath(path)
        if path not in _variants:
            _variants[path] = _open(path)
        return _variants[path]
    if _lib is not None:
        return _lib
    _lib = _open(LIB_PATH)
    return _lib


def _open(path):
    if not os.path.exists(path):
        raise OSError(f"{path} is missing: build it with `make -C {os.path.join(_HERE, 'csrc')} -j8` "
                      "(or __graft_entry__.build())")
    # RTLD_NOW: every HIP/RCCL symbol of the library (and of the runtime it
    # pulls in) binds at load time.  A process that imports torch afterwards
    # maps torch's bundled HIP runtime too; lazy binding could then resolve
    # some of our calls into that second runtime.
    lib = ctypes.CDLL(path, mode=os.RTLD_NOW | os.RTLD_LOCAL)
    P = ctypes.POINTER
    vp = ctypes.c_void_p
    sigs = {
        "bm_abi_version": ([], ctypes.c_int),
        "bm_strerror": ([ctypes.c_int], ctypes.c_char_p),
        "bm_device_count": ([P(ctypes.c_int)], ctypes.c_int),
        "bm_device_pci_bus_id": ([ctypes.c_int, ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
        "bm_ctx_create": ([ctypes.c_int, P(vp)], ctypes.c_int),
        "bm_ctx_create_devices": ([P(ctypes.c_int), ctypes.c_int, P(vp)], ctypes.c_int),
        "bm_ctx_destroy": ([vp], ctypes.c_int),
        "bm_ctx_num_devices": ([vp, P(ctypes.c_int)], ctypes.c_int),
        "bm_rccl_unique_id": ([ctypes.c_char_p], ctypes.c_int),
        "bm_ctx_create_rank": ([ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, P(vp)], ctypes.c_int),
        "bm_ctx_create_rank_local": ([ctypes.c_int, ctypes.c_int, ctypes.c_int, P(vp)], ctypes.c_int),
        "bm_ctx_join_rank": ([vp, ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
        "bm_ctx_leave_rank": ([vp], ctypes.c_int),
        "bm_ctx_rank_joined": ([vp, P(ctypes.c_int)], ctypes.c_int),
        "bm_ctx_set_peer_timeout": ([vp, ctypes.c_int], ctypes.c_int),
        "bm_ctx_set_test_rccl_fault": ([vp, ctypes.c_int], ctypes.c_int),
        "bm_ctx_set_test_start_delay": ([vp, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "bm_ctx_rank": ([vp, P(ctypes.c_int), P(ctypes.c_int)], ctypes.c_int),
        "bm_reduce_gpu": ([vp, P(Result), ctypes.c_size_t, P(Result)], ctypes.c_int),
        "bm_ctx_set_test_fault": ([vp, ctypes.c_int], ctypes.c_int),
        "bm_search_gpu": ([vp, ctypes.c_char_p, ctypes.c_size_t, c_u64, c_u64, P(Result)], ctypes.c_int),
        "bm_hash_gpu": ([vp, ctypes.c_char_p, ctypes.c_size_t, P(c_u64), ctypes.c_size_t, P(c_u64)],
                        ctypes.c_int),
        "bm_ctx_set_timing": ([vp, ctypes.c_int], ctypes.c_int),
        "bm_ctx_last_stats": ([vp, P(Stats)], ctypes.c_int),
        "bm_ctx_set_blocks_per_cu": ([vp, ctypes.c_int], ctypes.c_int),
        "bm_ctx_set_max_windows": ([vp, ctypes.c_int], ctypes.c_int),
        "bm_ctx_set_combine": ([vp, ctypes.c_int], ctypes.c_int),
        "bm_ctx_set_task_digits": ([vp, ctypes.c_int], ctypes.c_int),
        "bm_ctx_set_split": ([vp, P(ctypes.c_uint32), ctypes.c_int], ctypes.c_int),
        "bm_ctx_get_split": ([vp, P(ctypes.c_uint32), ctypes.c_int, P(ctypes.c_int)], ctypes.c_int),
        "bm_ctx_set_balance": ([vp, ctypes.c_int], ctypes.c_int),
        "bm_split_range": ([c_u64, c_u64, P(ctypes.c_uint32), ctypes.c_int, P(c_u64), P(c_u64)], ctypes.c_int),
        "bm_plan_segments": ([ctypes.c_char_p, ctypes.c_size_t, c_u64, c_u64, P(Segment), ctypes.c_int,
                              P(ctypes.c_int)], ctypes.c_int),
        "bm_plan_segments_ex": ([ctypes.c_char_p, ctypes.c_size_t, c_u64, c_u64, ctypes.c_int, P(Segment),
                                 ctypes.c_int, P(ctypes.c_int)], ctypes.c_int),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    # the stats structs above are this ABI's layout: any other build (an
    # older BTCMINER_LIB variant included) would be misread, so it is refused
    if lib.bm_abi_version() != BM_ABI_VERSION:
        raise OSError(f"{path}: ABI version {lib.bm_abi_version()}, expected {BM_ABI_VERSION}; rebuild it")
    return lib


def strerror(status):
    try:
        return load().bm_strerror(status).decode()
    except OSError:
        return f"status {status}"


def check(status, what):
    if status != BM_OK:
        raise BtcMinerError(status, what)


def device_count():
    n = ctypes.c_int(0)
    check(load().bm_device_count(ctypes.byref(n)), "bm_device_count")
    return n.value


def device_pci_bus_id(device: int) -> str:
    """PCI bus id of a visible device, e.g. "0000:05:00.0"."""
    buf = ctypes.create_string_buffer(64)
    check(load().bm_device_pci_bus_id(device, buf, len(buf)), "bm_device_pci_bus_id")
    return buf.value.decode()


DEFAULT_MAX_WINDOWS = 64


def plan_segments(msg: bytes, lower: int, upper: int, max_windows: int = DEFAULT_MAX_WINDOWS):
    """Host-side launch plan (pure CPU): list of Segment structs."""
    lib = load()
    n = ctypes.c_int(0)
    f = lib.bm_plan_segments_ex
    check(f(msg, len(msg), lower, upper, max_windows, None, 0, ctypes.byref(n)), "bm_plan_segments")
    arr = (Segment * max(n.value, 1))()
    check(f(msg, len(msg), lower, upper, max_windows, arr, n.value, ctypes.byref(n)), "bm_plan_segments")
    return list(arr[: n.value])


def split_range(lower: int, upper: int, n: int, shares=None):
    """The library's partitioner (bm_split_range, pure CPU): n inclusive
    pieces of [lower, upper], None for an empty one; shares None: near-equal."""
    lo, hi = (c_u64 * n)(), (c_u64 * n)()
    sh = (ctypes.c_uint32 * n)(*shares) if shares is not None else None
    check(load().bm_split_range(lower, upper, sh, n, lo, hi), "bm_split_range")
    return [(a, b) if a <= b else None for a, b in zip(lo, hi)]


def rccl_unique_id() -> bytes:
    """RCCL unique id for a process group (rank 0 makes it, every rank
    passes it to Context(rank=..., world=..., unique_id=...))."""
    buf = ctypes.create_string_buffer(BM_RCCL_ID_BYTES)
    check(load().bm_rccl_unique_id(buf), "bm_rccl_unique_id")
    return buf.raw


class Context:
    """Owns a bm_ctx over one or more GPUs.  Not thread-safe (like the C ctx).

    Context(devices=[...]) / Context(num_gpus=N): one process, N devices.
    Context(devices=[d], rank=r, world=w): rank r of w (one process per GPU)
    outside a group: search() scans rank r's piece and returns its partial;
    join(uid) then makes it a member of the RCCL group.
    Context(devices=[d], rank=r, world=w, unique_id=uid): both steps at once
    (blocks until all w ranks join)."""

    def __init__(self, devices=None, num_gpus=0, rank=None, world=None, unique_id=None, lib_path=None):
        lib = load(lib_path)
        h = ctypes.c_void_p()
        if world is not None:
            if devices is None or len(devices) != 1 or rank is None:
                raise ValueError("a rank context takes devices=[device], rank and world")
            if unique_id is None:
                check(lib.bm_ctx_create_rank_local(devices[0], rank, world, ctypes.byref(h)),
                      "bm_ctx_create_rank_local")
            else:
                if len(unique_id) != BM_RCCL_ID_BYTES:
                    raise ValueError(f"unique_id must be {BM_RCCL_ID_BYTES} bytes")
                check(lib.bm_ctx_create_rank(devices[0], rank, world, unique_id, ctypes.byref(h)),
                      "bm_ctx_create_rank")
        elif devices is not None:
            ids = (ctypes.c_int * len(devices))(*devices)
            check(lib.bm_ctx_create_devices(ids, len(devices), ctypes.byref(h)), "bm_ctx_create_devices")
        else:
            check(lib.bm_ctx_create(num_gpus, ctypes.byref(h)), "bm_ctx_create")
        self._lib = lib
        self._h = h

    @property
    def handle(self):
        if self._h is None:
            raise ValueError("context closed")
        return self._h

    def close(self):
        if self._h is not None:
            self._lib.bm_ctx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def num_devices(self):
        n = ctypes.c_int(0)
        check(self._lib.bm_ctx_num_devices(self.handle, ctypes.byref(n)), "bm_ctx_num_devices")
        return n.value

    def rank(self):
        """(rank, world) of the context's process group ((0, 1) if none)."""
        r, w = ctypes.c_int(0), ctypes.c_int(0)
        check(self._lib.bm_ctx_rank(self.handle, ctypes.byref(r), ctypes.byref(w)), "bm_ctx_rank")
        return r.value, w.value

    def join(self, unique_id: bytes, timeout_ms: int = 0):
        """Join the RCCL group (bm_ctx_join_rank): every rank, same id."""
        if len(unique_id) != BM_RCCL_ID_BYTES:
            raise ValueError(f"unique_id must be {BM_RCCL_ID_BYTES} bytes")
        check(self._lib.bm_ctx_join_rank(self.handle, unique_id, timeout_ms), "bm_ctx_join_rank")

    def leave(self):
        check(self._lib.bm_ctx_leave_rank(self.handle), "bm_ctx_leave_rank")

    def joined(self) -> bool:
        j = ctypes.c_int(0)
        check(self._lib.bm_ctx_rank_joined(self.handle, ctypes.byref(j)), "bm_ctx_rank_joined")
        return bool(j.value)

    def set_peer_timeout(self, timeout_ms: int):
        check(self._lib.bm_ctx_set_peer_timeout(self.handle, timeout_ms), "bm_ctx_set_peer_timeout")

    def set_test_rccl_fault(self, where: int):
        check(self._lib.bm_ctx_set_test_rccl_fault(self.handle, where), "bm_ctx_set_test_rccl_fault")

    def set_test_start_delay(self, device: int, delay_us: int):
        """Test hook: hold back device `device`'s submission by delay_us at
        the start of every later search (a late-starting GPU)."""
        check(self._lib.bm_ctx_set_test_start_delay(self.handle, device, delay_us), "bm_ctx_set_test_start_delay")

    def reduce(self, pairs):
        """Lexicographic min of (hash, nonce) pairs by the GPU reductions
        (bm_reduce_gpu, a test entry)."""
        n = len(pairs)
        arr = (Result * max(n, 1))(*[Result(h, nn) for h, nn in pairs])
        r = Result()
        check(self._lib.bm_reduce_gpu(self.handle, arr, n, ctypes.byref(r)), "bm_reduce_gpu")
        return r.hash, r.nonce

    def set_test_fault(self, launches: int):
        check(self._lib.bm_ctx_set_test_fault(self.handle, launches), "bm_ctx_set_test_fault")

    def search(self, msg: bytes, lower: int, upper: int):
        """Inclusive [lower, upper] min-scan -> (hash, nonce)."""
        r = Result()
        check(self._lib.bm_search_gpu(self.handle, msg, len(msg), lower, upper, ctypes.byref(r)), "bm_search_gpu")
        return r.hash, r.nonce

    def hash_many(self, msg: bytes, nonces):
        n = len(nonces)
        arr = (c_u64 * max(n, 1))(*nonces)
        out = (c_u64 * max(n, 1))()
        check(self._lib.bm_hash_gpu(self.handle, msg, len(msg), arr, n, out), "bm_hash_gpu")
        return list(out[:n])

    def set_timing(self, on: bool):
        check(self._lib.bm_ctx_set_timing(self.handle, 1 if on else 0), "bm_ctx_set_timing")

    def set_combine(self, mode: int):
        check(self._lib.bm_ctx_set_combine(self.handle, mode), "bm_ctx_set_combine")

    def set_task_digits(self, digits: int):
        check(self._lib.bm_ctx_set_task_digits(self.handle, digits), "bm_ctx_set_task_digits")

    def set_max_windows(self, n: int):
        check(self._lib.bm_ctx_set_max_windows(self.handle, n), "bm_ctx_set_max_windows")

    def set_blocks_per_cu(self, n: int):
        check(self._lib.bm_ctx_set_blocks_per_cu(self.handle, n), "bm_ctx_set_blocks_per_cu")

    def set_split(self, shares):
        """Integer shares, one per slot (devices, or ranks of the group; the
        same on every rank), for the range partitioner; None: near-equal."""
        shares = list(shares or [])
        arr = (ctypes.c_uint32 * max(len(shares), 1))(*shares)
        check(self._lib.bm_ctx_set_split(self.handle, arr, len(shares)), "bm_ctx_set_split")

    def get_split(self):
        """The shares the next search will use ([] when near-equal)."""
        n = ctypes.c_int(0)
        check(self._lib.bm_ctx_get_split(self.handle, None, 0, ctypes.byref(n)), "bm_ctx_get_split")
        arr = (ctypes.c_uint32 * max(n.value, 1))()
        check(self._lib.bm_ctx_get_split(self.handle, arr, n.value, ctypes.byref(n)), "bm_ctx_get_split")
        return list(arr[: n.value])

    def set_balance(self, on: bool):
        """Multi-device contexts: shares follow each device's measured rate."""
        check(self._lib.bm_ctx_set_balance(self.handle, 1 if on else 0), "bm_ctx_set_balance")

    def last_stats(self):
        s = Stats()
        check(self._lib.bm_ctx_last_stats(self.handle, ctypes.byref(s)), "bm_ctx_last_stats")
        return s
