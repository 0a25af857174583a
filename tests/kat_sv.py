"""Known-answer tests of the reference over test_data-sv.avro, transcribed with their sources.

Every expected value is copied from the reference's own tests; the segment list holds the same
segment twice and the broker merges two server copies, so every count/sum is 4x one segment
(BaseSingleValueQueriesTest.java:142, BaseQueriesTest.java:220-238).

Each entry: (query, expected rows, expected stats (numDocsScanned, numEntriesScannedPostFilter,
numTotalDocs), source).  numEntriesScannedInFilter is the reference's own iterator count (the docs its scan
iterators examine); it is checked separately, against the KAT's 63 064 per segment
(InnerSegmentAggregationSingleValueQueriesTest.java:56) and against oracle.filter_entries for every filter.
"""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "test_data_sv.npz")

# BaseSingleValueQueriesTest.java:99-107 (schema), :111-112 (inverted index columns)
DATA_TYPES = {
    "column1": "INT", "column3": "INT", "column5": "STRING", "column6": "INT", "column7": "INT",
    "column9": "INT", "column11": "STRING", "column12": "STRING", "column17": "INT", "column18": "INT",
    "daysSinceEpoch": "INT",
}
INVERTED = ("column6", "column7", "column11", "column17", "column18")

# BaseSingleValueQueriesTest.java:77-81
FILTER = (" WHERE column1 > 100000000"
          " AND column3 BETWEEN 20000000 AND 1000000000"
          " AND column5 = 'gFuH'"
          " AND (column6 < 500000000 OR column11 NOT IN ('t', 'P'))"
          " AND daysSinceEpoch = 126164076")
GROUP_BY = " GROUP BY column9 ORDER BY v1 DESC, v2 DESC LIMIT 1"  # InterSegmentAggregation...Test.java:39


def load_columns():
    z = np.load(GOLDEN, allow_pickle=False)
    return {c: (z[c], DATA_TYPES[c]) for c in DATA_TYPES}


_IA = "InterSegmentAggregationSingleValueQueriesTest.java"
_IG = "InterSegmentGroupBySingleValueQueriesTest.java"

KATS = [
    # ---- COUNT (:45-91)
    ("SELECT COUNT(*) FROM testTable", [[120000]], (120000, 0, 120000), _IA + ":48-54"),
    ("SELECT COUNT(*) FROM testTable" + FILTER, [[24516]], (24516, 0, 120000), _IA + ":56-58"),
    ("SELECT COUNT(*) FROM testTable GROUP BY column9 ORDER BY COUNT(*) DESC LIMIT 1", [[64420]],
     (120000, 120000, 120000), _IA + ":60-63"),
    ("SELECT COUNT(*) FROM testTable" + FILTER + " GROUP BY column9 ORDER BY COUNT(*) DESC LIMIT 1", [[17080]],
     (24516, 24516, 120000), _IA + ":65-67"),
    # ---- MAX (:93-117) -- the no-filter form is answered from metadata in the reference (0 post-filter)
    ("SELECT MAX(column1) AS v1, MAX(column3) AS v2 FROM testTable", [[2146952047.0, 2147419555.0]],
     (120000, 0, 120000), _IA + ":97-103"),
    ("SELECT MAX(column1) AS v1, MAX(column3) AS v2 FROM testTable" + FILTER, [[2146952047.0, 999813884.0]],
     (24516, 49032, 120000), _IA + ":105-108"),
    ("SELECT MAX(column1) AS v1, MAX(column3) AS v2 FROM testTable" + GROUP_BY, [[2146952047.0, 2146630496.0]],
     (120000, 360000, 120000), _IA + ":110-113"),
    ("SELECT MAX(column1) AS v1, MAX(column3) AS v2 FROM testTable" + FILTER + GROUP_BY,
     [[2146952047.0, 999813884.0]], (24516, 73548, 120000), _IA + ":115-118"),
    # ---- MIN (:120-147)
    ("SELECT MIN(column1) AS v1, MIN(column3) AS v2 FROM testTable", [[240528.0, 17891.0]],
     (120000, 0, 120000), _IA + ":124-131"),
    ("SELECT MIN(column1) AS v1, MIN(column3) AS v2 FROM testTable" + FILTER, [[101116473.0, 20396372.0]],
     (24516, 49032, 120000), _IA + ":133-136"),
    ("SELECT MIN(column1) AS v1, MIN(column3) AS v2 FROM testTable GROUP BY column9 ORDER BY v1, v2 LIMIT 1",
     [[240528.0, 17891.0]], (120000, 360000, 120000), _IA + ":138-142"),
    ("SELECT MIN(column1) AS v1, MIN(column3) AS v2 FROM testTable" + FILTER +
     " GROUP BY column9 ORDER BY v1, v2 LIMIT 1", [[101116473.0, 91804599.0]], (24516, 73548, 120000),
     _IA + ":144-147"),
    # ---- SUM (:149-175)
    ("SELECT SUM(column1) AS v1, SUM(column3) AS v2 FROM testTable", [[129268741751388.0, 129156636756600.0]],
     (120000, 240000, 120000), _IA + ":152-158"),
    ("SELECT SUM(column1) AS v1, SUM(column3) AS v2 FROM testTable" + FILTER,
     [[27503790384288.0, 12429178874916.0]], (24516, 49032, 120000), _IA + ":160-163"),
    ("SELECT SUM(column1) AS v1, SUM(column3) AS v2 FROM testTable" + GROUP_BY,
     [[69526727335224.0, 69225631719808.0]], (120000, 360000, 120000), _IA + ":165-168"),
    ("SELECT SUM(column1) AS v1, SUM(column3) AS v2 FROM testTable" + FILTER + GROUP_BY,
     [[19058003631876.0, 8606725456500.0]], (24516, 73548, 120000), _IA + ":170-173"),
    # ---- DISTINCTCOUNTHLL (:262-283)
    ("SELECT DISTINCTCOUNTHLL(column1) AS v1, DISTINCTCOUNTHLL(column3) AS v2 FROM testTable",
     [[5977, 23825]], (120000, 0, 120000), _IA + ":266-273"),
    ("SELECT DISTINCTCOUNTHLL(column1) AS v1, DISTINCTCOUNTHLL(column3) AS v2 FROM testTable" + FILTER,
     [[1886, 4492]], (24516, 49032, 120000), _IA + ":275-277"),
    ("SELECT DISTINCTCOUNTHLL(column1) AS v1, DISTINCTCOUNTHLL(column3) AS v2 FROM testTable" + GROUP_BY,
     [[3592, 11889]], (120000, 360000, 120000), _IA + ":279-280"),
    ("SELECT DISTINCTCOUNTHLL(column1) AS v1, DISTINCTCOUNTHLL(column3) AS v2 FROM testTable" + FILTER + GROUP_BY,
     [[1324, 3197]], (24516, 73548, 120000), _IA + ":282-283"),
    # ---- group-by order-by tables (InterSegmentGroupBySingleValueQueriesTest.java:62-140)
    ("SELECT column11, SUM(column1) FROM testTable GROUP BY column11 ORDER BY column11",
     [["", 5935285005452.0], ["P", 88832999206836.0], ["gFuH", 63202785888.0], ["o", 18105331533948.0],
      ["t", 16331923219264.0]], (120000, 240000, 120000), _IG + ":64-72"),
    ("SELECT column11, sum(column1) FROM testTable GROUP BY column11 ORDER BY column11 DESC",
     [["t", 16331923219264.0], ["o", 18105331533948.0], ["gFuH", 63202785888.0], ["P", 88832999206836.0],
      ["", 5935285005452.0]], (120000, 240000, 120000), _IG + ":74-78"),
    ("SELECT column11, column12, SUM(column1) FROM testTable GROUP BY column11, column12 ORDER BY column11, column12",
     [["", "HEuxNvH", 3789390396216.0], ["", "KrNxpdycSiwoRohEiTIlLqDHnx", 733802350944.0],
      ["", "MaztCmmxxgguBUxPti", 1333941430664.0], ["", "dJWwFk", 55470665124.0],
      ["", "oZgnrlDEtjjVpUoFLol", 22680162504.0], ["P", "HEuxNvH", 21998672845052.0],
      ["P", "KrNxpdycSiwoRohEiTIlLqDHnx", 18069909216728.0], ["P", "MaztCmmxxgguBUxPti", 27177029040008.0],
      ["P", "TTltMtFiRqUjvOG", 4462670055540.0], ["P", "XcBNHe", 120021767504.0]],
     (120000, 360000, 120000), _IG + ":87-98"),
    ("SELECT column11, column12, SUM(column1) FROM testTable"
     " GROUP BY column11, column12 ORDER BY column11, column12 LIMIT 15",
     [["", "HEuxNvH", 3789390396216.0], ["", "KrNxpdycSiwoRohEiTIlLqDHnx", 733802350944.0],
      ["", "MaztCmmxxgguBUxPti", 1333941430664.0], ["", "dJWwFk", 55470665124.0],
      ["", "oZgnrlDEtjjVpUoFLol", 22680162504.0], ["P", "HEuxNvH", 21998672845052.0],
      ["P", "KrNxpdycSiwoRohEiTIlLqDHnx", 18069909216728.0], ["P", "MaztCmmxxgguBUxPti", 27177029040008.0],
      ["P", "TTltMtFiRqUjvOG", 4462670055540.0], ["P", "XcBNHe", 120021767504.0],
      ["P", "dJWwFk", 6224665921376.0], ["P", "fykKFqiw", 1574451324140.0], ["P", "gFuH", 860077643636.0],
      ["P", "oZgnrlDEtjjVpUoFLol", 8345501392852.0], ["gFuH", "HEuxNvH", 29872400856.0]],
     (120000, 360000, 120000), _IG + ":100-109"),
    ("SELECT column11, column12, SUM(column1) FROM testTable"
     " GROUP BY column11, column12 ORDER BY column11, column12 DESC",
     [["", "oZgnrlDEtjjVpUoFLol", 22680162504.0], ["", "dJWwFk", 55470665124.0],
      ["", "MaztCmmxxgguBUxPti", 1333941430664.0], ["", "KrNxpdycSiwoRohEiTIlLqDHnx", 733802350944.0],
      ["", "HEuxNvH", 3789390396216.0], ["P", "oZgnrlDEtjjVpUoFLol", 8345501392852.0],
      ["P", "gFuH", 860077643636.0], ["P", "fykKFqiw", 1574451324140.0], ["P", "dJWwFk", 6224665921376.0],
      ["P", "XcBNHe", 120021767504.0]], (120000, 360000, 120000), _IG + ":111-121"),
    ("SELECT column11, column12, SUM(column1) FROM testTable GROUP BY column11, column12"
     " ORDER BY column11, sum(column1)",
     [["", "oZgnrlDEtjjVpUoFLol", 22680162504.0], ["", "dJWwFk", 55470665124.0],
      ["", "KrNxpdycSiwoRohEiTIlLqDHnx", 733802350944.0], ["", "MaztCmmxxgguBUxPti", 1333941430664.0],
      ["", "HEuxNvH", 3789390396216.0], ["P", "XcBNHe", 120021767504.0], ["P", "gFuH", 860077643636.0],
      ["P", "fykKFqiw", 1574451324140.0], ["P", "TTltMtFiRqUjvOG", 4462670055540.0],
      ["P", "dJWwFk", 6224665921376.0]], (120000, 360000, 120000), _IG + ":123-132"),
    ("SELECT sum(column1), MIN(column6) FROM testTable GROUP BY column11 ORDER BY column11",
     [[5935285005452.0, 2.96467636E8], [88832999206836.0, 1689277.0], [63202785888.0, 2.96467636E8],
      [18105331533948.0, 2.96467636E8], [16331923219264.0, 1980174.0]], (120000, 360000, 120000),
     _IG + ":156-163"),
    ("SELECT column12, MIN(column6) FROM testTable GROUP BY column12 ORDER BY Min(column6) DESC, column12",
     [["XcBNHe", 329467557.0], ["fykKFqiw", 296467636.0], ["gFuH", 296467636.0], ["HEuxNvH", 6043515.0],
      ["MaztCmmxxgguBUxPti", 6043515.0], ["dJWwFk", 6043515.0], ["KrNxpdycSiwoRohEiTIlLqDHnx", 1980174.0],
      ["TTltMtFiRqUjvOG", 1980174.0], ["oZgnrlDEtjjVpUoFLol", 1689277.0]], (120000, 240000, 120000),
     _IG + ":174-183"),
]

# Queries the reference answers from segment metadata (NonScanBasedAggregationOperator,
# AggregationPlanNode.java:108-119): no filter, no group-by, only MIN/MAX/COUNT/DISTINCTCOUNT* on
# dictionary columns.  Both paths report numDocsScanned = totalDocs and 0 post-filter entries.
