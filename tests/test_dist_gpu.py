"""The multi-GPU code path (RCCL process group, tree broadcast + unpack, ResultRing all-gathers, the sharded C4 / C5
helpers) on the box's one GPU, bit for bit against the one-process answers (tests/dist_child.py).

The child is launched by torch.distributed.run with one rank, so its first GPU work is the nccl initialisation, as in
a rank of bench.py's N > 1 run (the driver's 8-GPU node).  This module sorts before the other GPU test modules, so the
pytest process has not used the GPU when it starts the child (conftest.py counts devices without initialising HIP).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_collective_path_world1_bit_exact(tmp_path):
    out = tmp_path / "dist_report.json"
    env = dict(os.environ)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"  # dmabuf IPC, the only kind the box's driver supports
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dist_child.py"), str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, "child failed (%d):\n%s\n%s" % (r.returncode, r.stdout[-4000:], r.stderr[-4000:])
    rep = json.loads(out.read_text())
    assert rep["world"] == 1 and rep["backend"] == "nccl"
    assert rep["replica_is_new_handle"] and rep["replica_equal"]
    assert rep["replica_entry_cut"] == "built"  # the unpacked replica builds its own cut (derived data)
    assert rep["ring_batches_equal"] == [True, True, True]
    assert rep["narrow_batches_equal"] == [True, True, True]
    assert rep["rebuild_equal"] and rep["rebuild_no_face"]
    assert rep["visibility_equal"] and 0.05 < rep["visibility_visible_frac"] < 0.95
    assert rep["alongnormal_equal"] and rep["alongnormal_hit_frac"] > 0.9
    assert rep["c4_equal"] and rep["c4_dtypes"] == ["uint32", "uint32", "float64"]
