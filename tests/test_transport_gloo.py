"""Multi-process rank collectives over torch.distributed gloo (world_size 2 and 4, 127.0.0.1):
the host transport behind skm_build_set_transport and the exchange planning of a key-range pass
(send ranges from the owner-major bucket starts, the per-bucket count all-to-all, the receive
layout), on CPU; the whole multi-process build on one GPU (-m gpu)."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(mode, world, tmp_path, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "gloo_worker.py"), mode, str(tmp_path)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for k in range(world):
        assert (tmp_path / f"ok.{k}").exists(), r.stderr[-3000:]


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_transport_and_exchange_plan(skm, tmp_path, world):
    run_ranks("plan", world, tmp_path)


@pytest.mark.gpu
def test_gloo_two_process_build_matches_oracle(skm, gpu, tmp_path):
    run_ranks("build", 2, tmp_path, timeout=400)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_gloo_multi_process_matrix_matches_oracle(skm, gpu, tmp_path, world):
    """kmers-matrix-distance over `world` processes on one GPU: owner-partitioned hits and
    band-routed k-mer groups through the host transport, pairs bit-exact."""
    run_ranks("matrix", world, tmp_path, timeout=400)
