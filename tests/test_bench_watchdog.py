"""bench.py's N>1 watchdog (VERDICT r2 "what's weak" 2): a side leg stuck in
an exchange must end the run with a non-zero exit code and the stuck leg's
error in the printed JSON line -- never rc 0.  CPU only: two gloo ranks stuck
in a point-to-point exchange nobody completes (bench.py --watchdog-selftest)."""
import json
import os
import socket
import subprocess
import sys

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_watchdog_exits_nonzero_on_a_stuck_exchange():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(ROOT / "bench.py"), "--gpus", "2", "--watchdog-selftest", "--replica-timeout", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=env, cwd=str(ROOT))
    assert r.returncode != 0, f"watchdog run ended with rc 0:\n{r.stdout}\n{r.stderr}"
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert "timed out after 1.0 s" in line["replica_exchange"]["error"]
    assert line["watchdog"] == {"expired": True, "stage": "replica_exchange", "exit_code": 3}
    assert "exitcode  : 3" in r.stderr or "exit code 3" in r.stderr
