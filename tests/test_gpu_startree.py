"""GPU: queries answered from star-tree indexes (StarTreeV2; GroupByPlanNode.java:77-99, AggregationPlanNode.java:122-141,
StarTreeFilterOperator.java:157-358) through ph_segment_add_star_tree + ph_query_execute, against the oracle's
restatement (oracle/startree.py: traversal, remaining predicates, pair-column aggregation) segment by segment -- star
segments mixed with plain ones, every statistic -- and against the raw-document answer (skipStarTree / the oracle's
raw execution): COUNT / MIN / MAX bit-exact, SUM of the DOUBLE pair columns within 1e-9 relative (summation order)."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import startree as S
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from pinot_amd.startree import attach
from tests.test_gpu_parity import rows_equal
from tests.test_startree_cpu import STAR_QUERIES, make_star, star_table

pytestmark = pytest.mark.gpu
RTOL = 1e-9


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd.engine import GpuContext
    c = GpuContext(0)
    yield c
    c.close()


def _segments(ctx, seed, sizes=(6000, 2500, 3001), max_leaf=10, star=(True, True, False)):
    rng = np.random.default_rng(seed)
    gpu, ora = [], []
    for i, (n, has) in enumerate(zip(sizes, star)):
        cols = star_table(rng, n)
        seg, st, oseg, osd = make_star(cols, name=f"st{i}", max_leaf=max_leaf)
        p = ctx.pin(seg)
        if has:
            attach(p, st)
        gpu.append(p)
        ora.append((oseg, osd if has else None))
    return gpu, ora


def _check(ctx, gpu, ora, sql):
    q = parse_sql(sql)
    r = ctx.execute(q, gpu)
    keys, aggs, stats, served = S.execute_with_star_trees(q, ora)
    got = reduce_groups(q, r.keys, r.aggs)
    exp = reduce_groups(q, keys, aggs)
    rows_equal(got.rows, exp.rows, RTOL)
    assert r.stats.num_segments_star_tree == served, sql
    assert r.stats.num_docs_scanned == stats["num_docs_scanned"], sql
    assert r.stats.num_total_docs == stats["num_total_docs"], sql
    assert r.stats.num_entries_scanned_post_filter == stats["num_entries_scanned_post_filter"], sql
    assert r.stats.num_entries_scanned_in_filter == stats["num_entries_scanned_in_filter"], sql
    # the raw documents give the same answer
    raw = O.execute(q, [o for o, _ in ora])
    rows_equal(got.rows, reduce_groups(q, raw.keys, raw.aggs).rows, RTOL)
    return r, served


@pytest.mark.parametrize("sql", STAR_QUERIES)
@pytest.mark.parametrize("max_leaf", [3, 25])
def test_star_tree_queries(ctx, sql, max_leaf):
    gpu, ora = _segments(ctx, len(sql) + max_leaf, max_leaf=max_leaf)
    _, served = _check(ctx, gpu, ora, sql)
    if "'zz'" not in sql:
        assert served == 2


@pytest.mark.parametrize("sql", STAR_QUERIES[:4])
def test_star_tree_only_segments(ctx, sql):
    gpu, ora = _segments(ctx, 11, sizes=(4000, 5000), star=(True, True))
    r, served = _check(ctx, gpu, ora, sql)
    assert served == 2 and r.stats.num_segments_processed == 2


def test_skip_star_tree_and_not_fit(ctx):
    gpu, ora = _segments(ctx, 21)
    for sql in ["SET skipStarTree=true; SELECT d1, COUNT(*), SUM(m) FROM t GROUP BY d1",
                "SELECT z, COUNT(*) FROM t GROUP BY z",
                "SELECT COUNT(*) FROM t WHERE NOT d1 = 10",
                "SELECT COUNT(*) FROM t WHERE d1 = 10 OR d2 = 'ca'",
                "SELECT MAX(m), MIN(m) FROM t"]:
        _, served = _check(ctx, gpu, ora, sql)
        assert served == 0, sql


def test_star_tree_random_filters(ctx):
    rng = np.random.default_rng(77)
    gpu, ora = _segments(ctx, 31, sizes=(8000, 3000, 2000), max_leaf=6)
    for _ in range(12):
        conj = []
        if rng.random() < 0.7:
            conj.append(f"d1 IN ({', '.join(str(10 * int(x)) for x in rng.integers(0, 6, 2))})")
        if rng.random() < 0.6:
            conj.append(f"d2 {'=' if rng.random() < .5 else '<>'} '{['ca', 'ny', 'tx', 'wa'][rng.integers(0, 4)]}'")
        if rng.random() < 0.6:
            lo = int(rng.integers(0, 30)) * 1000
            conj.append(f"(d3 BETWEEN {lo} AND {lo + 9000} OR d3 = 39007)")
        where = (" WHERE " + " AND ".join(conj)) if conj else ""
        gb = ["", "d1", "d2", "d3", "d1, d3"][rng.integers(0, 5)]
        sel = (gb + ", " if gb else "") + "COUNT(*), SUM(m), MIN(m), MAX(x)"
        sql = f"SELECT {sel} FROM t{where}" + (f" GROUP BY {gb}" if gb else "")
        _check(ctx, gpu, ora, sql)


def test_star_tree_multi_device_and_trim(ctx):
    from pinot_amd.engine import GpuContext
    rng_seed = 41
    m = GpuContext(devices=[0, 0])
    try:
        gpu, ora = _segments(m, rng_seed)
        for sql in STAR_QUERIES[1:5]:
            _check(m, gpu, ora, sql)
        # segment group trim runs one segment per call: each takes its own star-tree
        q = parse_sql("SET minSegmentGroupTrimSize=1; SELECT d3, COUNT(*) FROM t GROUP BY d3 ORDER BY COUNT(*) DESC, "
                      "d3 LIMIT 3")
        r = m.execute(q, gpu)
        assert r.stats.num_segments_star_tree == 2
    finally:
        m.close()


def test_filter_execute_ignores_star_tree(ctx):
    # FilterPlanNode's operator is over the segment's own documents: ph_filter_execute never takes the star-tree
    gpu, ora = _segments(ctx, 51, sizes=(5000,), star=(True,))
    q = parse_sql("SELECT COUNT(*) FROM t WHERE d1 = 20 AND d2 = 'ny'")
    words, cnt, st = ctx.filter(q, gpu[0])
    mask, _ = O.filter_docs(q, ora[0][0])
    assert cnt == int(mask.sum()) and st.num_total_docs == 5000


def test_star_tree_from_segment_directory(ctx, tmp_path):
    # ph_segment_load_dir reads v3/star_tree_index + star_tree_index_map + the startree.v2.* metadata
    # (StarTreeLoaderUtils.loadStarTreeV2) and takes the tree like a pinned one
    from tests import segment_dirs as SD
    rng = np.random.default_rng(91)
    cols = star_table(rng, 7000)
    seg, st, oseg, osd = make_star(cols, name="sd", max_leaf=5)
    path = str(tmp_path / "st")
    SD.write_v3(seg, path)
    SD.write_star_trees(path, [st])
    loaded = ctx.load_segment_dir(path)
    from pinot_amd import native as N
    assert N.lib().ph_segment_num_star_trees(loaded.handle) == 1
    for sql in STAR_QUERIES:
        _check(ctx, [loaded], [(oseg, osd)], sql)
