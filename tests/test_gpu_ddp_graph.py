"""The multi-rank graph-mode training step on a real GPU: two `gloo` ranks sharing cuda:0
(tests/ddp_graph_worker.py) run the Trainer's split graphs -- forward + backward with the
in-graph bucket events, the bucket all-reduces on the side stream behind them, the optimiser
graph -- as the driver's N > 1 bench does over RCCL.  Replicas fed different batches must stay
bit-identical; losses finite; the capture must have happened."""
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


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [2])
def test_split_graph_step_two_ranks_one_gpu(ranks):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "ddp_graph_worker.py")]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "OK" in r.stdout, out[-3000:]
    assert f"world {ranks} split True" in r.stdout, out[-3000:]
