"""The RCCL ("nccl") branch of distributed.py on the GPU: a one-rank process group over RCCL
runs the end-of-run collectives the OOS batch uses (all-gather of per-vintage summaries,
all-reduce SUM / MAX, the log-mean-exp of log scores) with device tensors, and their results
equal the single-process values.  (The GPU box has one GPU; the world-2 path is covered by the
gloo tests in test_distributed.py.)"""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_nccl_world1_collectives():
    code = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {str(ROOT)!r})
        import numpy as np
        import __graft_entry__
        dm = __graft_entry__.load_package().distributed
        dist, w = dm.init("nccl", min_world=1)
        assert dist is not None and dist.get_backend() == "nccl", dist
        assert dm._device_for(dist).type == "cuda"
        local = {{u: np.full(3, float(u)) for u in (4, 1, 7)}}
        g = dm.gather_summaries(dist, local, None)
        assert list(g) == [1, 4, 7] and all(np.array_equal(g[u], local[u]) for u in g)
        a = np.arange(6.0).reshape(2, 3)
        assert np.array_equal(dm.allreduce_sum(dist, a), a)
        assert dm.max_over_ranks(dist, 2.5) == 2.5
        x = np.random.default_rng(3).normal(size=40)
        m = x.max()
        ref = m + np.log(np.mean(np.exp(x - m)))
        assert abs(dm.logmeanexp_over_ranks(dist, x) - ref) < 1e-14
        dist.barrier()
        dist.destroy_process_group()
        print("nccl world-1 ok")
    """)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=150)
    print(r.stdout[-2000:], r.stderr[-3000:])
    assert r.returncode == 0 and "nccl world-1 ok" in r.stdout
