"""Shared fixtures.  `-m gpu` tests need a gfx950 device and call the
product through the C ABI (libbtcminer.so); everything else runs on CPU.
The CPU oracle (oracle/) is used here only as the checker."""
import ctypes
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
U64 = (1 << 64) - 1


def pytest_configure(config):
    # libbtcminer.so binds to /opt/rocm's HIP runtime; torch bundles its own.
    # Keep torch out of this process so only one runtime is mapped (bench.py
    # does the same: its ranks meet over a file rendezvous, not torch).
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")


CONFIG_TAG = re.compile(r"\[(C[1-5])\]")


def pytest_collection_modifyitems(config, items):
    """Run order: README's known answers, then the BASELINE config tests
    (ids tagged [C1]..[C5]: whole-range C1/C2/C3, C4's whole 2^40 range, C5
    at size), then the rest, and the bench / torchrun subprocess rehearsals
    last -- so a run cut short still pins every config."""
    def rank(item):
        if item.name.startswith("test_readme_known_answers"):
            return (0, "")
        m = CONFIG_TAG.search(item.nodeid)
        if m:
            return (1, m.group(1))
        if any(k in item.name for k in ("bench", "torchrun", "rehears")):
            return (3, "")
        return (2, "")
    items.sort(key=rank)


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


class Oracle:
    """ctypes view of oracle/liboracle.so (test infrastructure)."""

    def __init__(self, path):
        lib = ctypes.CDLL(path)
        u64, P = ctypes.c_uint64, ctypes.POINTER
        lib.oracle_hash.argtypes = [ctypes.c_char_p, ctypes.c_size_t, u64]
        lib.oracle_hash.restype = u64
        lib.oracle_search.argtypes = [ctypes.c_char_p, ctypes.c_size_t, u64, u64, P(u64), P(u64)]
        lib.oracle_search_excl.argtypes = lib.oracle_search.argtypes
        lib.oracle_search_mt.argtypes = [ctypes.c_char_p, ctypes.c_size_t, u64, u64, ctypes.c_int, ctypes.c_int,
                                         P(u64), P(u64)]
        lib.oracle_search_mt.restype = ctypes.c_int
        lib.oracle_search_x16.argtypes = [ctypes.c_char_p, ctypes.c_size_t, u64, u64, ctypes.c_int, P(u64), P(u64)]
        lib.oracle_search_x16.restype = ctypes.c_int
        self.lib = lib

    def hash(self, msg: bytes, nonce: int) -> int:
        return self.lib.oracle_hash(msg, len(msg), nonce)

    def search(self, msg: bytes, lo: int, hi: int, threads: int = 1, openssl: bool = False, go_shape: bool = False):
        """go_shape: OpenSSL with hash.go's per-call allocations (use_openssl = 2)."""
        h, n = ctypes.c_uint64(), ctypes.c_uint64()
        if threads == 1 and not openssl and not go_shape:
            self.lib.oracle_search(msg, len(msg), lo, hi, ctypes.byref(h), ctypes.byref(n))
        else:
            mode = 2 if go_shape else 1 if openssl else 0
            assert self.lib.oracle_search_mt(msg, len(msg), lo, hi, threads, mode,
                                             ctypes.byref(h), ctypes.byref(n)) == 0
        return h.value, n.value

    def search_x16(self, msg: bytes, lo: int, hi: int, threads: int = 8):
        """16-lane AVX-512 scan (oracle/bm_scan16.c): golden answers over long
        ranges only, itself checked against search() (tests/test_oracle.py)."""
        h, n = ctypes.c_uint64(), ctypes.c_uint64()
        rc = self.lib.oracle_search_x16(msg, len(msg), lo, hi, threads, ctypes.byref(h), ctypes.byref(n))
        if rc == -2:
            raise OSError("oracle_search_x16 needs AVX-512F")
        assert rc == 0
        return h.value, n.value

    def search_excl(self, msg: bytes, lo: int, hi: int):
        h, n = ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.oracle_search_excl(msg, len(msg), lo, hi, ctypes.byref(h), ctypes.byref(n))
        return h.value, n.value


@pytest.fixture(scope="session")
def oracle():
    path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(path):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    return Oracle(path)


@pytest.fixture(scope="session")
def gpu_ctx():
    from distributed_bitcoin_minter_amd import Context
    ctx = Context(num_gpus=1)
    yield ctx
    ctx.close()
