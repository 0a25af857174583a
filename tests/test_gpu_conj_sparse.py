"""GPU parity of the register-direct scan-AND front end of the sparse kernels (conj_reg.h): k_group_sparse and
k_agg_sparse over segments filtered by ANDs of dictId scan leaves only (AndDocIdSet over ScanBasedFilterOperators,
SSB on dictionary-encoded dimensions).  The leaves are decoded 32 docs per lane straight from the packed streams and
only the matched docs' keys and values are gathered; results and every statistic (numEntriesScannedInFilter
included) against the oracle.  Covered: range / IN / NOT IN leaves, sets staged in LDS (<= 8192 ids) and read from HBM
(larger), leaf columns over 16 bits (32-byte lane loads), 2-operand value terms, segments that end mid-step, and the
plan picked by the selectivity estimate as well as forced (PH_GROUP_SPARSE / PH_AGG_SPARSE), in the default leaf-by-leaf
load form and the all-leaves-at-once one (PH_SPARSE_C=2, leaves <= 8 bits)."""
import numpy as np
import pytest

from pinot_amd.engine import SCAN_KERNEL_NAMES
from tests.seeds import seed_of
from tests.test_gpu_parity import _both, ctx  # noqa: F401  (the module's context fixture)

pytestmark = pytest.mark.gpu

SIZES = (20_000, 4095, 64 * 300 + 1, 100_003)


def _table(rng, n):
    return {
        "x": (rng.integers(0, 7, n).astype(np.int32), "INT"),
        "y": (rng.integers(0, 300, n).astype(np.int32), "INT"),
        "z": (rng.integers(0, 20_000, n).astype(np.int32), "INT"),       # set leaves beyond the LDS-staged size
        "w": (rng.integers(0, 1 << 18, n).astype(np.int32), "INT"),      # an 18-bit leaf column
        "g1": (rng.integers(0, 50, n).astype(np.int32), "INT"),
        "g2": (rng.integers(0, 40, n).astype(np.int32), "INT"),
        "m": (rng.integers(-50_000, 50_000, n).astype(np.int32), "INT"),
        "p": (rng.integers(1, 11, n).astype(np.int32), "INT"),
        "d": (np.round(rng.normal(0, 100, n), 2), "DOUBLE"),
    }


WHERES = [
    "x = 3 AND y < 40",
    "x IN (1, 5) AND y BETWEEN 10 AND 200 AND g2 <> 7",
    "y < 20 AND z IN (5, 77, 1234, 19999, 8000, 8191, 8192, 12345)",
    "z NOT IN (3, 4, 5) AND x = 0 AND y >= 290",
    "w < 2000 AND x <> 2",
    "w BETWEEN 100000 AND 101000 AND y < 150 AND x IN (0, 6) AND g1 < 25",
    "x = 9 AND y = 1",  # no doc matches
]


@pytest.mark.parametrize("force", [False, True, "wide"])
@pytest.mark.parametrize("where", WHERES)
def test_conj_sparse_group_by(ctx, monkeypatch, where, force):  # noqa: F811
    if force:
        monkeypatch.setenv("PH_GROUP_SPARSE", "1")
    if force == "wide":
        monkeypatch.setenv("PH_SPARSE_C", "2")
    rng = np.random.default_rng(seed_of("conj-g" + where))
    tables = [_table(rng, n) for n in SIZES]
    for group in ("g1", "g1, g2", "y, g2"):
        r, _ = _both(ctx, tables, f"SET numGroupsLimit=10000000; SELECT {group}, COUNT(*), SUM(m), MIN(m), MAX(m) "
                                  f"FROM t WHERE {where} GROUP BY {group} ORDER BY {group} LIMIT 100000")
        if force and "x = 9" not in where:
            assert SCAN_KERNEL_NAMES[r.stats.scan_kernel] == "k_group_sparse", (where, group)
        _both(ctx, tables, f"SET numGroupsLimit=10000000; SELECT {group}, SUM(m * p), SUM(m - p) FROM t "
                           f"WHERE {where} GROUP BY {group} ORDER BY {group} LIMIT 100000")


@pytest.mark.parametrize("force", [False, True, "wide"])
@pytest.mark.parametrize("where", WHERES)
def test_conj_sparse_aggregation(ctx, monkeypatch, where, force):  # noqa: F811
    if force:
        monkeypatch.setenv("PH_AGG_SPARSE", "1")
    if force == "wide":
        monkeypatch.setenv("PH_SPARSE_C", "2")
    rng = np.random.default_rng(seed_of("conj-a" + where))
    tables = [_table(rng, n) for n in SIZES]
    for sel in ("SUM(m * p)", "SUM(m - p)", "SUM(m), MIN(m), MAX(m)", "SUM(d), MIN(d), MAX(d)", "SUM(m + d)"):
        r, _ = _both(ctx, tables, f"SELECT {sel} FROM t WHERE {where}")
        if force and "x = 9" not in where:
            assert SCAN_KERNEL_NAMES[r.stats.scan_kernel] == "k_agg_sparse", (where, sel)
