"""GPU: k_and_dfa / k_and_compose (numEntriesScannedInFilter of an AND of scans, and_walk.h) through the test hooks
phx_and_walk_entries_device / phx_and_walk_tables_host: the device's workgroup tables and entries against the host's
composition of the same chunk tables and against the iterator simulation, on random leaves, and the longest walk a chunk can
take (every doc a match of 12 scans), which must finish within a stated bound (a chunk's walks are bounded by its 128-512
docs: there is no rerun cliff) (AndDocIdIterator.java:40-72, SVScanDocIdIterator.java:101-112)."""
import ctypes
import time

import numpy as np
import pytest

from pinot_amd import native as N
from tests.test_filter_sim_cpu import _bitmap, _native_sim, _scan_and

pytestmark = pytest.mark.gpu


def _device(docs, n, gtab=None):
    f = N.lib().phx_and_walk_entries_device
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p]
    bits = np.concatenate([_bitmap(d, n) for d in docs])
    return f(bits.ctypes.data, len(docs), n, gtab.ctypes.data if gtab is not None else None)


def _host_tables(docs, n, block):
    f = N.lib().phx_and_walk_tables_host
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]
    bits = np.concatenate([_bitmap(d, n) for d in docs])
    k = len(docs)
    cw = N.lib().phx_and_dfa_chunk_words()  # the chunk size the device uses (words of 64 docs)
    ng = ((n + 64 * cw - 1) // (64 * cw) + block - 1) // block
    t = np.zeros(2 * (k + 1) * ng, np.uint32)
    assert f(bits.ctypes.data, k, n, block, t.ctypes.data) == ng
    return t, ng


@pytest.mark.parametrize("seed", range(24))
def test_device_tables_match_host(seed):
    rng = np.random.default_rng(9100 + seed)
    n = int(rng.choice([1, 63, 64, 511, 513, 4097, 131_072, 200_001, 1_000_003]))
    k = int(rng.integers(2, 13))
    dens = rng.choice([0.003, 0.02, 0.15, 0.5, 0.9, 1.0], size=k)
    docs = [rng.random(n) < d for d in dens]
    block = 128 if k <= 8 else 64
    exp_t, ng = _host_tables(docs, n, block)
    got_t = np.zeros_like(exp_t)
    got = _device(docs, n, got_t)
    k1 = k + 1
    for part, name in ((0, "delta"), (1, "exit")):
        a = exp_t[part * k1 * ng:(part + 1) * k1 * ng].reshape(k1, ng)
        b = got_t[part * k1 * ng:(part + 1) * k1 * ng].reshape(k1, ng)
        bad = np.argwhere(a != b)
        assert bad.size == 0, (name, seed, n, k, bad[:5].tolist(), a[tuple(bad[0])], b[tuple(bad[0])])
    root, leaves = _scan_and(k)
    assert got == _native_sim(root, leaves, docs, n), (seed, n, k)


def test_worst_case_is_bounded():
    # every doc matches all 12 scans: every chunk walks one epoch per doc of 12 advance() calls (the longest walk a chunk can
    # take); the sum has a closed form, numDocs x k (k calls per doc, the last epoch at numDocs included), and 2^24
    # docs must finish within 2 s
    n, k = 1 << 24, 12
    docs = [np.ones(n, bool)] * k
    t0 = time.time()
    got = _device(docs, n)
    dt = time.time() - t0
    assert got == n * k
    assert dt < 2.0, dt
