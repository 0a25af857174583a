"""Tuning aid: epochs the AND-walk automaton (and_walk.h dfa_chunk) spends per 256-doc chunk on the SSB scan flight's
leaves -- the type -1 walk against the other entry types' walks (which stop at the first of the type -1 walk's first
kDfaHist candidates they reach).  python3 tools/dfa_epochs.py [docs] [hist]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LEAVES = {
    "Q1.1": ["d_year = 1993", "lo_discount BETWEEN 1 AND 3", "lo_quantity < 25"],
    "Q1.2": ["d_yearmonthnum = 199401", "lo_discount BETWEEN 4 AND 6", "lo_quantity BETWEEN 26 AND 35"],
    "Q1.3": ["d_weeknuminyear = 6", "d_year = 1994", "lo_discount BETWEEN 5 AND 7", "lo_quantity BETWEEN 26 AND 35"],
    "Q2.1": ["p_category = 'MFGR#12'", "s_region = 'AMERICA'"],
    "Q2.2": ["p_brand1 BETWEEN 'MFGR#2221' AND 'MFGR#2228'", "s_region = 'ASIA'"],
    "Q2.3": ["p_brand1 = 'MFGR#2239'", "s_region = 'EUROPE'"],
    "Q3.1": ["c_region = 'ASIA'", "s_region = 'ASIA'", "d_year BETWEEN 1992 AND 1997"],
    "Q3.2": ["c_nation = 'UNITED STATES'", "s_nation = 'UNITED STATES'", "d_year BETWEEN 1992 AND 1997"],
    "Q3.3": ["c_city IN ('UNITED KI1', 'UNITED KI5')", "s_city IN ('UNITED KI1', 'UNITED KI5')",
             "d_year BETWEEN 1992 AND 1997"],
    "Q3.4": ["c_city IN ('UNITED KI1', 'UNITED KI5')", "s_city IN ('UNITED KI1', 'UNITED KI5')",
             "d_yearmonthnum = 199712"],
    "Q4.1": ["c_region = 'AMERICA'", "s_region = 'AMERICA'", "p_mfgr IN ('MFGR#1', 'MFGR#2')"],
    "Q4.2": ["c_region = 'AMERICA'", "s_region = 'AMERICA'", "d_year IN (1997, 1998)", "p_mfgr IN ('MFGR#1', 'MFGR#2')"],
    "Q4.3": ["s_nation = 'UNITED STATES'", "d_year IN (1997, 1998)", "p_category = 'MFGR#14'"],
}


def walk_chunk(S, c0, c1, hist):
    """dfa_chunk's epochs: (type -1 epochs, other types' epochs, per-type epoch counts)."""
    k = len(S)

    def f_of(M):
        f = 0
        while f < k and S[f][M]:
            f += 1
        return f

    def nxt(i, x):
        while x < c1:
            if S[i][x]:
                return x
            x += 1
        return -1

    def step(M):
        f = f_of(M)
        if f == k:
            return M + 1 if M + 1 < c1 else -1
        return nxt(f, M + 1)
    seen = []
    M, n0 = c0, 0
    while M >= 0:
        if len(seen) < hist:
            seen.append(M)
        n0 += 1
        M = step(M)
    others = []
    for e in range(k):
        M, ne = nxt(e, c0), 0
        while M >= 0:
            ne += 1
            if M in seen:
                break
            M = step(M)
        others.append(ne)
    return n0, others


def main():
    from bench import oracle_segments
    from oracle import oracle as O
    from pinot_amd.query import parse_sql
    from tests import workloads as W
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    hist = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    seg = oracle_segments([W.ssb_segment_buffers("e", n, seed=0xC004)])[0]
    tot0 = toto = 0
    for name, leaves in LEAVES.items():
        S = [O.filter_docs(parse_sql(f"SELECT COUNT(*) FROM lineorder WHERE {w}"), seg)[0] for w in leaves]
        S = [list(map(bool, s)) for s in S]
        a = b = 0
        worst = 0
        per = np.zeros(len(S))
        for c0 in range(0, n, 256):
            n0, oth = walk_chunk(S, c0, min(n, c0 + 256), hist)
            a += n0
            b += sum(oth)
            per += oth
            worst = max(worst, n0 + sum(oth))
        ch = (n + 255) // 256
        dens = [f"{np.mean(s):.3f}" for s in S]
        print(f"{name} k={len(S)} dens {dens} per chunk: type-1 {a / ch:6.1f} others {b / ch:6.1f} "
              f"({', '.join(f'{x / ch:.1f}' for x in per)}) worst {worst}", flush=True)
        tot0 += a
        toto += b
    print(f"flight: type-1 {tot0} others {toto}")


if __name__ == "__main__":
    main()
