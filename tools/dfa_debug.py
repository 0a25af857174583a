"""Debug: device vs host DFA workgroup tables on small inputs (GPU box)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tests.test_gpu_and_walk import _device, _host_tables
for n, k, seed in ((600, 2, 1), (64, 2, 2), (1, 2, 3), (4097, 4, 4), (513, 3, 5)):
    rng = np.random.default_rng(seed)
    docs = [rng.random(n) < 0.5 for _ in range(k)]
    exp_t, ng = _host_tables(docs, n, 256)
    got_t = np.zeros_like(exp_t)
    got = _device(docs, n, got_t)
    k1 = k + 1
    print(n, k, "host delta", exp_t[:k1 * ng].reshape(k1, ng)[:, 0].tolist(), "exit", exp_t[k1 * ng:].reshape(k1, ng)[:, 0].tolist())
    print(n, k, "dev  delta", got_t[:k1 * ng].reshape(k1, ng)[:, 0].tolist(), "exit", got_t[k1 * ng:].reshape(k1, ng)[:, 0].tolist(), "entries", got)
