"""CPU sanitizer run of the host parsers: tests/sanitize/fuzz_host.cpp, built with
-fsanitize=address,undefined over loader.cpp / rawfwd.cpp / roaring.cpp, parses every seed of a corpus written here
(raw chunk forward indexes in every codec and writer version, roaring inverted indexes with and without run
containers, V3 and V1 segment directories, the reference's own startree index_map) and seeded corruptions of each
(truncations, bit flips, extreme 32-bit fields, zeroed spans).  Every corrupted input must come back as a status code
(ph::Error) with no sanitizer report; any report aborts the harness (-fno-sanitize-recover=all)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from pinot_amd.segment import build_inverted_index, create_segment, write_raw_forward_index
from tests import segment_dirs as SD

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "build", "sanitize", "fuzz_host")
REF_INDEX_MAP = os.path.join(ROOT, "tests", "golden", "startree_segment", "index_map")
TYPES = {"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32, "DOUBLE": np.float64}


def _corpus(tmp):
    rng = np.random.default_rng(91)
    lines = []
    for dt, npt in TYPES.items():
        n = 2345
        v = (rng.integers(-1000, 1000, n) if dt in ("INT", "LONG") else np.round(rng.normal(0, 50, n), 2)).astype(npt)
        v[: n // 8] = v[0]  # runs: overlapping LZ4 / Snappy copies
        for comp in ("PASS_THROUGH", "LZ4", "LZ4_LENGTH_PREFIXED", "SNAPPY"):
            for version in (2, 3, 4):
                p = os.path.join(tmp, f"raw_{dt}_{comp}_{version}.bin")
                write_raw_forward_index(v, dt, comp, version, docs_per_chunk=300).tofile(p)
                lines.append(f"raw {p} {dt} {n}")
    for run_opt in (False, True):
        n, card = 200_000, 9
        ids = np.sort(rng.integers(0, card, n)) if run_opt else rng.integers(0, card, n)
        ids[:card] = np.arange(card)
        p = os.path.join(tmp, f"inv_{int(run_opt)}.bin")
        np.asarray(build_inverted_index(ids.astype(np.int32), card, run_opt)).tofile(p)
        lines.append(f"inv {p} {card}")
    m = 3000
    cols = {"a": (rng.integers(0, 40, m).astype(np.int32), "INT"),
            "s.t": (np.sort(rng.integers(0, 9, m)).astype(np.int32), "INT"),
            "l": (rng.integers(-10**9, 10**9, m).astype(np.int64), "LONG"),
            "str": (np.array(["x", "yy", ""])[rng.integers(0, 3, m)], "STRING")}
    buf = create_segment("fz", cols, inverted=("a",))
    SD.write_v3(buf, os.path.join(tmp, "v3seg"))
    SD.write_v1(buf, os.path.join(tmp, "v1seg"))
    lines += [f"dir {os.path.join(tmp, 'v3seg')}", f"dir {os.path.join(tmp, 'v1seg')}",
              f"map {os.path.join(tmp, 'v3seg', 'v3', 'index_map')}", f"map {REF_INDEX_MAP}"]
    manifest = os.path.join(tmp, "manifest.txt")
    with open(manifest, "w") as f:
        f.write("\n".join(lines) + "\n")
    return manifest


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with the sanitizer runtimes")
def test_host_parsers_under_asan_ubsan(tmp_path):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "sanitize")], check=True, timeout=600)
    manifest = _corpus(str(tmp_path))
    scratch = tmp_path / "scratch"
    scratch.mkdir()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([HARNESS, manifest, str(scratch), "150"], capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "no sanitizer report" in r.stdout
    print(r.stdout.strip())
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc with the sanitizer runtimes")
def test_oracle_thread_pool_under_tsan():
    # the CPU restatement's multi-threaded combine (or_execute's worker pool) under ThreadSanitizer
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "sanitize")], check=True, timeout=600)
    r = subprocess.run([os.path.join(ROOT, "build", "sanitize", "tsan_oracle")], capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0, (r.stdout, r.stderr[-4000:])
    assert "equals the 1-thread run" in r.stdout and "ThreadSanitizer" not in r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with the sanitizer runtimes")
def test_library_host_concurrency_under_tsan():
    # the library's own host threads (host_pool.h) -- the filter statistic's simulation pool over
    # filter_sim.cpp and multi.cpp's per-device phases with a stub transport -- under ThreadSanitizer
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "sanitize")], check=True, timeout=600)
    r = subprocess.run([os.path.join(ROOT, "build", "sanitize", "tsan_host")], capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0, (r.stdout, r.stderr[-4000:])
    assert "equal the 1-thread run" in r.stdout and "exception rethrown" in r.stdout, r.stdout
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
