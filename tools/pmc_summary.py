"""Summarise rocprofv3 PMC passes (tools/gpu_pmc.sh) into HBM bytes per query for bench.py's roofline.traffic.

FETCH_SIZE / WRITE_SIZE are per-dispatch kilobytes (rocprofv3 derived counters over TCC_EA0_RDREQ/_WRREQ).
Per MI355X_MICROARCH.md ("HBM"), on gfx950 FETCH_SIZE reports half the bytes of wide 16-byte-per-lane streaming
reads, which is how the scan kernels read; it is doubled here ("fetch_corrected").  The bench ran two queries
(warmup + step), so totals over the scan-path kernels are halved to one query.
    python3 tools/pmc_summary.py <workload> <pmc dir> <out.json>
"""
import csv
import glob
import json
import os
import sys

# per-query kernels (one-time per-column caches -- k_encode_values, k_hll_table -- and pin-time fills excluded)
SCAN_KERNELS = ("k_scan", "k_part_scan", "k_part_reg", "k_part_agg", "k_agg", "k_group", "k_count_reg", "k_merge_overflow",
                "k_compact", "k_roaring")
# kernels that read with 16-byte-per-lane streaming loads: their FETCH_SIZE is doubled (gfx950 correction); the
# gathers (k_agg_sparse, k_roaring_or, k_compact_*) are reported as counted
STREAMING = ("k_scan", "k_part_scan", "k_part_agg", "k_agg_lean", "k_group_lds")
# register-direct kernels (k_part_reg, k_count_reg, k_agg_reg, k_group_reg): 16 B per lane at a lane stride of 4b
# bytes -- an access width the guide leaves uncalibrated, so their factor is calibrated on config 2, whose
# k_count_reg reads exactly the 2 500 000 000 stream bytes (REG_FACTOR env, default 2 = the streaming rule)
REG = ("k_part_reg", "k_count_reg", "k_agg_reg", "k_group_reg")


def totals(d, counter):
    per_kernel = {}
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if not any(k in name for k in SCAN_KERNELS):
                continue
            if row.get("Counter_Name") != counter:
                continue
            per_kernel[name] = per_kernel.get(name, 0.0) + float(row.get("Counter_Value", 0) or 0)
    return per_kernel


def main():
    w, d, out = sys.argv[1:4]
    fetch = totals(d, "FETCH_SIZE")
    write = totals(d, "WRITE_SIZE")
    queries = 2
    f_kb = sum(fetch.values()) / queries
    w_kb = sum(write.values()) / queries
    reg_factor = float(os.environ.get("REG_FACTOR", "2"))

    def factor(name):
        if any(k in name for k in REG):
            return reg_factor
        return 2 if any(k in name for k in STREAMING) else 1
    f_corr = sum(v * factor(name) for name, v in fetch.items()) / queries
    res = {
        "workload": w,
        "fetch_size_kb_per_query": f_kb,
        "write_size_kb_per_query": w_kb,
        "fetch_corrected_bytes": f_corr * 1024,
        "write_bytes": w_kb * 1024,
        "hbm_bytes_per_query": f_corr * 1024 + w_kb * 1024,
        "per_kernel_fetch_kb": {k: v / queries for k, v in fetch.items()},
        "per_kernel_write_kb": {k: v / queries for k, v in write.items()},
        "reg_factor": reg_factor,
        "note": "FETCH_SIZE of the 16-B/lane streaming kernels doubled (MI355X_MICROARCH.md gfx950 correction); "
                "register-direct kernels x reg_factor (calibrated on config 2's k_count_reg); gather kernels as "
                "counted; one-time column caches and pin-time fills excluded",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if not k.startswith("per_")}))


if __name__ == "__main__":
    main()
