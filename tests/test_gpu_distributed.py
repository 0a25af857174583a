"""GPU: the multi-GPU combine end to end through libpinot_hip at world size 2 -- two ranks sharing
cuda:0 over gloo (the GPU box has one GPU; RCCL needs one GPU per rank), each running ph_query_execute_dense ->
reduce_tables -> ph_dense_finalize on its own segments, compared on rank 0 with the oracle over all segments
(tests/dist_gpu_worker.py): the config-3 shape split into key-range shards, a DOUBLE SUM group-by, and config 5's
DISTINCTCOUNTHLL register max all-reduce.

The ranks are started by torch.distributed.run in a child process (the test process itself has initialised the GPU
and must not exec)."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_dense_partials_match_oracle(tmp_path):
    out = tmp_path / "result.txt"
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["OMP_NUM_THREADS"] = env.get("OMP_NUM_THREADS", "4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_gpu_worker.py"), str(out)]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert out.read_text().startswith("OK"), out.read_text()
