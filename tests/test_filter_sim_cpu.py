"""CPU: numEntriesScannedInFilter by iterator simulation.  The library's host simulator (filter_sim.cpp, reached
through the test hook phx_filter_entries_sim; the product calls it for filter shapes without a device pass) is checked
against the oracle's restatement of the reference iterators (oracle.filter_entries_of) on random filter trees and doc
sets, and the oracle's restatement against a fully literal variant (every next() batch by batch, no drain shortcut).
ANDs of scans only are summed by the leap-frog's per-chunk transition tables (and_walk.h: k_and_dfa / k_and_compose
on the device); the same tables run on the host through phx_and_walk_entries and are checked against the simulation
here at chunk sizes from 1 doc to one whole segment (exact at every size: no speculation), and on the GPU in
test_gpu_parity.py."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd import native as N

KINDS = {"scan": 0, "sorted": 1, "inverted": 2, "range": 2}
PRIO = {"sorted": 0, "range": 200, "scan": 500, "inverted": 10000}


def _random_tree(rng, depth, leaves):
    if depth == 0 or rng.random() < 0.35:
        kind = rng.choice(["scan", "scan", "scan", "sorted", "inverted", "range"])
        node = O._Leaf("leaf", len(leaves), None, kind == "scan")
        node.ikind = kind
        leaves.append(node)
        return node
    op = rng.choice(["and", "and", "or", "not"])
    node = O._Leaf(op)
    if op == "not":
        node.children = [_random_tree(rng, depth - 1, leaves)]
    else:
        node.children = [_random_tree(rng, depth - 1, leaves) for _ in range(int(rng.integers(2, 4)))]
    return node


def _docs(rng, n, kind):
    if kind == "sorted":  # a doc range
        a = int(rng.integers(0, n))
        b = int(rng.integers(a, n + 1))
        d = np.zeros(n, bool)
        d[a:b] = True
        return d
    return rng.random(n) < rng.choice([0.02, 0.2, 0.5, 0.9])


def _flatten(root):
    """The test hook's flat tree: rows (op, priority, leaf, first child, child count); a node's children are
    consecutive rows (a child's own subtree lives further on)."""
    out = []

    def rec(x, pos):
        if x.kind == "leaf":
            out[pos] = [0, PRIO[x.ikind], x.col_index, 0, 0]
            return
        op = {"and": 1, "or": 2, "not": 3}[x.kind]
        first = len(out)
        out.extend([None] * len(x.children))
        out[pos] = [op, 300 if op == 1 else 400, -1, first, len(x.children)]
        for j, c in enumerate(x.children):
            rec(c, first + j)

    out.append(None)
    rec(root, 0)
    return np.array(out, dtype=np.int32).ravel()


def _bitmap(d, n):
    nw = (n + 63) // 64
    padded = np.zeros(nw * 64, bool)
    padded[:n] = d
    return np.packbits(padded.reshape(-1, 8)[:, ::-1], axis=1).ravel().view(np.uint64).copy()


def _walk(docs, n, shift):
    f = N.lib().phx_and_walk_entries
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32]
    bits = np.concatenate([_bitmap(d, n) for d in docs])
    return f(bits.ctypes.data, len(docs), n, shift)


def _native_sim(root, leaves, docs, n):
    L = N.lib()
    f = L.phx_filter_entries_sim
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64]
    flat = _flatten(root)
    kinds = np.array([KINDS[l.ikind] for l in leaves], dtype=np.int32)
    bits = [_bitmap(d, n) for d in docs]
    ptrs = (ctypes.c_void_p * len(bits))(*[b.ctypes.data for b in bits])
    return f(flat.ctypes.data, len(flat) // 5, kinds.ctypes.data, ptrs, len(bits), n)


class _LiteralScan(O._ScanIt):
    """SVScanDocIdIterator.next() batch by batch (no jump over empty batches), drained by next() calls."""

    def next(self):
        if self.cursor >= self.first_mismatch:
            while True:
                limit = min(self.n - self.next_doc, 256)
                if limit <= 0:
                    self.batch, self.cursor, self.first_mismatch = self.pos[:0], 0, 0
                    return O.EOF_DOC
                lo, hi = self.next_doc, self.next_doc + limit
                b = self.pos[np.searchsorted(self.pos, lo):np.searchsorted(self.pos, hi)]
                self.next_doc += limit
                self.entries += limit
                if len(b):
                    break
            self.batch, self.cursor, self.first_mismatch = b, 0, len(b)
        self.cursor += 1
        return int(self.batch[self.cursor - 1])

    def drain(self):
        while self.next() != O.EOF_DOC:
            pass


@pytest.mark.parametrize("seed", range(40))
def test_native_filter_sim_matches_oracle(seed):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.choice([1, 63, 64, 257, 3000, 20_011]))
    leaves = []
    root = _random_tree(rng, 3, leaves)
    docs = [_docs(rng, n, l.ikind) for l in leaves]
    exp = O.filter_entries_of(root, n, lambda node: docs[node.col_index])
    got = _native_sim(root, leaves, docs, n)
    assert got == exp, (seed, n)


@pytest.mark.parametrize("seed", range(15))
def test_oracle_sim_matches_literal_batches(seed, monkeypatch):
    rng = np.random.default_rng(2000 + seed)
    n = int(rng.choice([300, 5000]))
    leaves = []
    root = _random_tree(rng, 3, leaves)
    docs = [_docs(rng, n, l.ikind) for l in leaves]
    exp = O.filter_entries_of(root, n, lambda node: docs[node.col_index])
    monkeypatch.setattr(O, "_ScanIt", _LiteralScan)
    assert O.filter_entries_of(root, n, lambda node: docs[node.col_index]) == exp


def test_scan_and_closed_cases():
    # AND of scans only (AndDocIdIterator): hand-checked small cases
    n = 10
    a = np.zeros(n, bool)
    b = np.zeros(n, bool)
    a[[2, 5, 7]] = True
    b[[5, 7, 9]] = True
    la, lb = O._Leaf("leaf", 0, None, True), O._Leaf("leaf", 1, None, True)
    la.ikind = lb.ikind = "scan"
    root = O._Leaf("and")
    root.children = [la, lb]
    # next() #1 from 0: a.adv(0) -> 2 [3 docs]; b.adv(2) -> 5 [4]; a.adv(5) -> 5 [1]; output 5
    # next() #2 from 6: a.adv(6) -> 7 [2]; b.adv(7) -> 7 [1]; output 7
    # next() #3 from 8: a.adv(8) -> EOF [2 docs: 8, 9]
    assert O.filter_entries_of(root, n, lambda x: [a, b][x.col_index]) == 3 + 4 + 1 + 2 + 1 + 2
    assert _native_sim(root, [la, lb], [a, b], n) == 13
    assert _walk([a, b], n, 30) == 13
    assert _walk([a, b], n, 2) in (13, -1)


def _scan_and(k):
    root = O._Leaf("and")
    leaves = []
    for i in range(k):
        leaf = O._Leaf("leaf", i, None, True)
        leaf.ikind = "scan"
        leaves.append(leaf)
    root.children = leaves
    return root, leaves


@pytest.mark.parametrize("seed", range(30))
def test_and_walk_matches_simulation(seed):
    rng = np.random.default_rng(3000 + seed)
    n = int(rng.choice([1, 2, 64, 65, 4095, 4097, 20_000, 70_001]))
    k = int(rng.integers(2, 6))
    dens = rng.choice([0.003, 0.02, 0.15, 0.5, 0.9, 1.0], size=k)
    docs = [rng.random(n) < d for d in dens]
    root, leaves = _scan_and(k)
    exp = _native_sim(root, leaves, docs, n)
    assert exp == O.filter_entries_of(root, n, lambda x: docs[x.col_index])
    assert _walk(docs, n, 62) == exp  # one chunk: the plain walk
    for shift in (0, 1, 3, 6, 8, 9, 10, 12):
        assert _walk(docs, n, shift) == exp, (seed, shift)


def test_and_walk_at_bench_densities():
    # SSB-like densities at the product's 512-doc chunks (and 64-doc ones): the composed tables are exact
    rng = np.random.default_rng(7)
    n = 200_000
    for dens in ([1 / 7, 3 / 11, 0.48], [1 / 84, 3 / 11, 0.2], [2 / 250, 2 / 250, 6 / 7], [1 / 25, 1 / 5],
                 [5e-4, 0.5], [1e-5, 0.5, 0.5], [0.5, 1e-5], [1 / 5, 1 / 5, 2 / 7, 2 / 5],
                 [2 / 250, 2 / 250, 1 / 84]):
        docs = [rng.random(n) < d for d in dens]
        root, leaves = _scan_and(len(dens))
        exp = _native_sim(root, leaves, docs, n)
        assert _walk(docs, n, 9) == exp, dens
        assert _walk(docs, n, 6) == exp, dens


def _walk_words(docs, n, width):
    f = N.lib().phx_and_walk_entries_words
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32]
    bits = np.concatenate([_bitmap(d, n) for d in docs])
    return f(bits.ctypes.data, len(docs), n, width)


@pytest.mark.parametrize("seed", range(30))
def test_and_walk_word_tables(seed):
    # k_and_dfa_reg's per-word tables (dfa_word: the type -1 walk's candidates as a mask, the other entry types
    # joining it through the epoch-sum bit planes), narrower ANDs padded with all-ones scans up to `width`
    rng = np.random.default_rng(4000 + seed)
    n = int(rng.choice([1, 2, 63, 64, 65, 127, 4097, 20_000, 70_001]))
    k = int(rng.integers(1, 5))
    dens = rng.choice([0.003, 0.02, 0.15, 0.5, 0.9, 1.0], size=k)
    docs = [rng.random(n) < d for d in dens]
    root, leaves = _scan_and(k)
    exp = _native_sim(root, leaves, docs, n) if k > 1 else _walk(docs, n, 62)
    for width in range(max(2, k), 5):
        assert _walk_words(docs, n, width) == exp, (seed, k, width)


def test_and_walk_word_tables_at_bench_densities():
    rng = np.random.default_rng(8)
    n = 100_000
    for dens in ([1 / 7, 3 / 11, 0.48], [1 / 84, 3 / 11, 0.2], [2 / 250, 2 / 250, 6 / 7], [1 / 25, 1 / 5],
                 [1 / 5, 1 / 5, 2 / 7, 2 / 5], [1.0, 1.0, 1.0, 1.0], [0.0, 1.0], [1.0, 0.0, 0.5]):
        docs = [rng.random(n) < d for d in dens]
        root, leaves = _scan_and(len(dens))
        exp = _native_sim(root, leaves, docs, n)
        assert _walk_words(docs, n, len(dens)) == exp, dens
        assert _walk_words(docs, n, 4) == exp, dens
