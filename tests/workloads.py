"""Synthetic data of the BASELINE.json configurations, shared by the GPU parity tests and bench.py.

Test infrastructure: generates column VALUES with seeded PCG64 generators; segments are then built by
pinot_amd.segment.create_segment (GPU) and oracle.build_segment (CPU checker) from the same values.

* config 1 -- README AdAnalytics (README.md:82-88): daysSinceEpoch sorted, accountId Zipf with 123456789 as the
  rank-1 id, clicks / impressions metrics.
* config 5 -- DISTINCTCOUNTHLL(u) over an inverted-index IN filter on c; u uniform over 2^27 user ids (b = 24 at
  >= ~8.5M rows per segment).
* config 4 -- SSB lineorder, denormalised (the flat table Pinot's SSB setups use): d_*, c_*, s_*, p_* dimension
  attributes plus lo_* metrics drawn from the SSB specification's domains (dbgen is not in the image).
"""
from __future__ import annotations

import numpy as np

# ------------------------------------------------------------------ config 1
ADS_SQL = ("SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM AdAnalyticsTable "
           "WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) "
           "GROUP BY daysSinceEpoch ORDER BY daysSinceEpoch LIMIT 100")


def ads_columns(n: int, seed: int = 0xAD01):
    rng = np.random.default_rng(seed)
    days = np.sort(rng.integers(17800, 17900, n)).astype(np.int32)
    # Zipf(s = 1.2) over 100 000 account ids; rank 1 is 123456789
    ranks = rng.zipf(1.2, n)
    ranks = np.where(ranks > 100_000, 1 + (ranks % 100_000), ranks)
    ids = np.where(ranks == 1, 123456789, 1_000_000 + ranks * 7).astype(np.int32)
    return {
        "daysSinceEpoch": (days, "INT"),
        "accountId": (ids, "INT"),
        "clicks": (rng.integers(0, 1001, n).astype(np.int32), "INT"),
        "impressions": (rng.integers(0, 100_001, n).astype(np.int32), "INT"),
    }


# ------------------------------------------------------------------ config 5
def hll_columns(n: int, seed: int = 0xC005, c_card: int = 1000):
    rng = np.random.default_rng(seed)
    return {
        "u": (rng.integers(0, 1 << 27, n).astype(np.int32), "INT"),
        "c": (rng.integers(0, c_card, n).astype(np.int32), "INT"),
    }


def hll_sql(ids, log2m=None):
    arg = "u" if log2m is None else f"u, {log2m}"
    return f"SELECT DISTINCTCOUNTHLL({arg}) FROM t WHERE c IN ({', '.join(str(i) for i in ids)})"


# ------------------------------------------------------------------ config 4 (SSB)
REGIONS = ["AFRICA", "AMERICA", "ASIA", "EUROPE", "MIDDLE EAST"]
NATIONS = [  # (nation, region index) -- TPC-H / SSB nation table
    ("ALGERIA", 0), ("ARGENTINA", 1), ("BRAZIL", 1), ("CANADA", 1), ("EGYPT", 4), ("ETHIOPIA", 0),
    ("FRANCE", 3), ("GERMANY", 3), ("INDIA", 2), ("INDONESIA", 2), ("IRAN", 4), ("IRAQ", 4), ("JAPAN", 2),
    ("JORDAN", 4), ("KENYA", 0), ("MOROCCO", 0), ("MOZAMBIQUE", 0), ("PERU", 1), ("CHINA", 2), ("ROMANIA", 3),
    ("SAUDI ARABIA", 4), ("VIETNAM", 2), ("RUSSIA", 3), ("UNITED KINGDOM", 3), ("UNITED STATES", 1),
]
MONTHS = ["Jan", "Feb", "Mar", "Apr", "May", "Jun", "Jul", "Aug", "Sep", "Oct", "Nov", "Dec"]


def _city(nation: str, k: np.ndarray) -> np.ndarray:
    # SSB city = first 9 characters of the nation name, space padded, + one digit (UNITED KI1 ... UNITED ST9)
    pre = (nation + " " * 9)[:9]
    return np.array([pre + str(int(d)) for d in k])


def ssb_columns(n: int, seed: int = 0xC004):
    """One denormalised lineorder segment of n rows."""
    rng = np.random.default_rng(seed)
    # dates: 1992-01-01 .. 1998-12-31 (SSB date dimension, 7 years)
    day = rng.integers(0, 2557, n)
    base = np.datetime64("1992-01-01")
    dates = base + day.astype("timedelta64[D]")
    years = dates.astype("datetime64[Y]").astype(np.int64) + 1970
    months = dates.astype("datetime64[M]").astype(np.int64) % 12 + 1
    doy = (dates - dates.astype("datetime64[Y]")).astype(np.int64)
    cols = {
        "d_year": (years.astype(np.int32), "INT"),
        "d_yearmonthnum": ((years * 100 + months).astype(np.int32), "INT"),
        "d_weeknuminyear": ((doy // 7 + 1).astype(np.int32), "INT"),
    }
    nat_names = np.array([x[0] for x in NATIONS])
    nat_region = np.array([REGIONS[x[1]] for x in NATIONS])
    for pfx in ("c", "s"):
        nat = rng.integers(0, 25, n)
        digit = rng.integers(0, 10, n)
        cities = np.array([(nm + " " * 9)[:9] for nm in nat_names], dtype=object)[nat] + digit.astype(str)
        cols[f"{pfx}_region"] = (nat_region[nat], "STRING")
        cols[f"{pfx}_nation"] = (nat_names[nat], "STRING")
        cols[f"{pfx}_city"] = (cities.astype(str), "STRING")
    mfgr = rng.integers(1, 6, n)
    cat = rng.integers(1, 6, n)
    brand = rng.integers(1, 41, n)
    cols["p_mfgr"] = (np.char.add("MFGR#", mfgr.astype(str)), "STRING")
    cols["p_category"] = (np.char.add("MFGR#", (mfgr * 10 + cat).astype(str)), "STRING")
    cols["p_brand1"] = (np.char.add("MFGR#", (mfgr * 1000 + cat * 100 + brand).astype(str)), "STRING")
    qty = rng.integers(1, 51, n)
    price = rng.integers(90_000, 200_001, n)  # p_retailprice in cents
    disc = rng.integers(0, 11, n)
    ext = qty * price // 100
    cols["lo_quantity"] = (qty.astype(np.int32), "INT")
    cols["lo_discount"] = (disc.astype(np.int32), "INT")
    cols["lo_extendedprice"] = (ext.astype(np.int32), "INT")
    cols["lo_revenue"] = ((ext * (100 - disc) // 100).astype(np.int32), "INT")
    cols["lo_supplycost"] = ((price * 6 // 1000).astype(np.int32), "INT")
    return cols


# The 13 SSB queries over the flat lineorder table (SSB specification; Q3.4's d_yearmonth 'Dec1997' as
# d_yearmonthnum 199712).  Q1.x / Q4.x aggregate 2-operand expressions.
SSB_QUERIES = {
    "Q1.1": "SELECT SUM(lo_extendedprice * lo_discount) AS revenue FROM lineorder WHERE d_year = 1993 "
            "AND lo_discount BETWEEN 1 AND 3 AND lo_quantity < 25",
    "Q1.2": "SELECT SUM(lo_extendedprice * lo_discount) AS revenue FROM lineorder WHERE d_yearmonthnum = 199401 "
            "AND lo_discount BETWEEN 4 AND 6 AND lo_quantity BETWEEN 26 AND 35",
    "Q1.3": "SELECT SUM(lo_extendedprice * lo_discount) AS revenue FROM lineorder WHERE d_weeknuminyear = 6 "
            "AND d_year = 1994 AND lo_discount BETWEEN 5 AND 7 AND lo_quantity BETWEEN 26 AND 35",
    "Q2.1": "SELECT d_year, p_brand1, SUM(lo_revenue) FROM lineorder WHERE p_category = 'MFGR#12' "
            "AND s_region = 'AMERICA' GROUP BY d_year, p_brand1 ORDER BY d_year, p_brand1 LIMIT 10000",
    "Q2.2": "SELECT d_year, p_brand1, SUM(lo_revenue) FROM lineorder WHERE p_brand1 BETWEEN 'MFGR#2221' "
            "AND 'MFGR#2228' AND s_region = 'ASIA' GROUP BY d_year, p_brand1 ORDER BY d_year, p_brand1 LIMIT 10000",
    "Q2.3": "SELECT d_year, p_brand1, SUM(lo_revenue) FROM lineorder WHERE p_brand1 = 'MFGR#2239' "
            "AND s_region = 'EUROPE' GROUP BY d_year, p_brand1 ORDER BY d_year, p_brand1 LIMIT 10000",
    "Q3.1": "SELECT c_nation, s_nation, d_year, SUM(lo_revenue) AS revenue FROM lineorder WHERE c_region = 'ASIA' "
            "AND s_region = 'ASIA' AND d_year >= 1992 AND d_year <= 1997 GROUP BY c_nation, s_nation, d_year "
            "ORDER BY d_year ASC, revenue DESC LIMIT 10000",
    "Q3.2": "SELECT c_city, s_city, d_year, SUM(lo_revenue) AS revenue FROM lineorder "
            "WHERE c_nation = 'UNITED STATES' AND s_nation = 'UNITED STATES' AND d_year >= 1992 AND d_year <= 1997 "
            "GROUP BY c_city, s_city, d_year ORDER BY d_year ASC, revenue DESC LIMIT 10000",
    "Q3.3": "SELECT c_city, s_city, d_year, SUM(lo_revenue) AS revenue FROM lineorder "
            "WHERE (c_city = 'UNITED KI1' OR c_city = 'UNITED KI5') AND (s_city = 'UNITED KI1' OR "
            "s_city = 'UNITED KI5') AND d_year >= 1992 AND d_year <= 1997 GROUP BY c_city, s_city, d_year "
            "ORDER BY d_year ASC, revenue DESC LIMIT 10000",
    "Q3.4": "SELECT c_city, s_city, d_year, SUM(lo_revenue) AS revenue FROM lineorder "
            "WHERE (c_city = 'UNITED KI1' OR c_city = 'UNITED KI5') AND (s_city = 'UNITED KI1' OR "
            "s_city = 'UNITED KI5') AND d_yearmonthnum = 199712 GROUP BY c_city, s_city, d_year "
            "ORDER BY d_year ASC, revenue DESC LIMIT 10000",
    "Q4.1": "SELECT d_year, c_nation, SUM(lo_revenue - lo_supplycost) AS profit FROM lineorder "
            "WHERE c_region = 'AMERICA' AND s_region = 'AMERICA' AND (p_mfgr = 'MFGR#1' OR p_mfgr = 'MFGR#2') "
            "GROUP BY d_year, c_nation ORDER BY d_year, c_nation LIMIT 10000",
    "Q4.2": "SELECT d_year, s_nation, p_category, SUM(lo_revenue - lo_supplycost) AS profit FROM lineorder "
            "WHERE c_region = 'AMERICA' AND s_region = 'AMERICA' AND (d_year = 1997 OR d_year = 1998) "
            "AND (p_mfgr = 'MFGR#1' OR p_mfgr = 'MFGR#2') GROUP BY d_year, s_nation, p_category "
            "ORDER BY d_year, s_nation, p_category LIMIT 10000",
    "Q4.3": "SELECT d_year, s_city, p_brand1, SUM(lo_revenue - lo_supplycost) AS profit FROM lineorder "
            "WHERE s_nation = 'UNITED STATES' AND (d_year = 1997 OR d_year = 1998) AND p_category = 'MFGR#14' "
            "GROUP BY d_year, s_city, p_brand1 ORDER BY d_year, s_city, p_brand1 LIMIT 10000",
}
SSB_INVERTED = ("c_region", "s_region", "c_nation", "s_nation", "c_city", "s_city", "p_mfgr", "p_category",
                "p_brand1")


def ssb_segment_buffers(name: str, n: int, seed: int = 0xC004, inverted=()):
    """A denormalised lineorder segment of n rows built straight in dictionary-id form (no string arrays of n
    entries): the same column set, value domains and dictionaries as ``ssb_columns`` (sorted distinct values),
    drawn from its own seeded PCG64 stream.  For bench-sized segments (10M rows in seconds; ~2 s more per inverted
    column); columns not in `inverted` have no inverted index, so their predicates run as dictId scans."""
    from pinot_amd.segment import SegmentBuffers, create_column, create_column_from_dict_ids
    rng = np.random.default_rng(seed)
    seg = SegmentBuffers(name, n)

    def put(col, dictionary, ids, dt):
        dictionary = np.asarray(dictionary)
        used = np.zeros(len(dictionary), bool)
        used[np.unique(ids)] = True  # dictionary = values present (sorted), ids renumbered
        remap = np.cumsum(used) - 1
        seg.columns[col] = create_column_from_dict_ids(col, dictionary[used], remap[ids].astype(np.int32), dt,
                                                       inverted=col in inverted, allow_sorted=False)
    day = rng.integers(0, 2557, n)
    base = np.datetime64("1992-01-01")
    all_days = base + np.arange(2557).astype("timedelta64[D]")
    yr = all_days.astype("datetime64[Y]").astype(np.int64) + 1970
    mo = all_days.astype("datetime64[M]").astype(np.int64) % 12 + 1
    wk = (all_days - all_days.astype("datetime64[Y]")).astype(np.int64) // 7 + 1
    ym = yr * 100 + mo
    for col, per_day in (("d_year", yr), ("d_yearmonthnum", ym), ("d_weeknuminyear", wk)):
        dic, inv = np.unique(per_day, return_inverse=True)
        put(col, dic.astype(np.int32), inv.reshape(-1)[day], "INT")
    nat_names = [x[0] for x in NATIONS]
    regions = sorted(REGIONS)
    nations = sorted(nat_names)
    cities = sorted({(nm + " " * 9)[:9] + str(d) for nm in nat_names for d in range(10)})
    region_of = np.array([regions.index(REGIONS[x[1]]) for x in NATIONS])
    nation_rank = np.array([nations.index(nm) for nm in nat_names])
    city_rank = np.array([[cities.index((nm + " " * 9)[:9] + str(d)) for d in range(10)] for nm in nat_names])
    for pfx in ("c", "s"):
        nat = rng.integers(0, 25, n)
        digit = rng.integers(0, 10, n)
        put(f"{pfx}_region", np.array(regions), region_of[nat], "STRING")
        put(f"{pfx}_nation", np.array(nations), nation_rank[nat], "STRING")
        put(f"{pfx}_city", np.array(cities), city_rank[nat, digit], "STRING")
    mfgr = rng.integers(1, 6, n)
    cat = rng.integers(1, 6, n)
    brand = rng.integers(1, 41, n)
    put("p_mfgr", np.array([f"MFGR#{i}" for i in range(1, 6)]), mfgr - 1, "STRING")
    cats = [m * 10 + c for m in range(1, 6) for c in range(1, 6)]
    put("p_category", np.array([f"MFGR#{v}" for v in cats]), (mfgr - 1) * 5 + (cat - 1), "STRING")
    brands = [m * 1000 + c * 100 + b for m in range(1, 6) for c in range(1, 6) for b in range(1, 41)]
    put("p_brand1", np.array([f"MFGR#{v}" for v in brands]), ((mfgr - 1) * 5 + (cat - 1)) * 40 + (brand - 1), "STRING")
    qty = rng.integers(1, 51, n)
    price = rng.integers(90_000, 200_001, n)
    disc = rng.integers(0, 11, n)
    ext = qty * price // 100
    for col, v in (("lo_quantity", qty), ("lo_discount", disc), ("lo_extendedprice", ext),
                   ("lo_revenue", ext * (100 - disc) // 100), ("lo_supplycost", price * 6 // 1000)):
        seg.columns[col] = create_column(col, v.astype(np.int32), "INT")
    return seg
