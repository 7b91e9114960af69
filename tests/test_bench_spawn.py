"""bench.py --gpus N without a launcher (VERDICT r3 "next" 1): the parent
starts the N rank processes itself (subprocesses, never exec, no GPU call in
the parent), relays rank 0's line and fails the run if any rank fails --
a multi-GPU request must never come back as a one-rank line.  CPU only:
the ranks join a gloo group (bench.py --plumbing-selftest)."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def _run(*extra, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--dist-backend", "gloo", "--plumbing-selftest", *extra]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=str(ROOT))


def test_gpus_2_spawns_two_ranks():
    r = _run("--gpus", "2")
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    # and nothing else on stdout: gloo's connection log and other library
    # prints go to stderr (bench.claim_stdout), so a driver can take stdout whole
    assert r.stdout.strip().splitlines() == lines, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert line["rccl"]["world_size"] == 2 and line["rccl"]["backend"] == "gloo"
    ranks = line["rccl"]["ranks"]
    assert [x["rank"] for x in ranks] == [0, 1]
    assert all(x["spawned_by_bench"] for x in ranks)
    assert len({x["pid"] for x in ranks}) == 2     # two processes, not one


def test_gpus_4_spawns_four_ranks():
    r = _run("--gpus", "4")
    assert r.returncode == 0, r.stderr
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert line["rccl"]["world_size"] == 4 and len({x["pid"] for x in line["rccl"]["ranks"]}) == 4


def test_a_failing_rank_fails_the_run():
    # rank 1 exits right after joining; rank 0 would wait forever in the
    # gather: the parent must stop it and report the failure, with no line
    r = _run("--gpus", "2", "--selftest-fail-rank", "1")
    assert r.returncode == 7, (r.returncode, r.stderr)
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")], r.stdout
    assert "rank 1 exited with code 7" in r.stderr


def test_launcher_world_size_mismatch_is_an_error():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--plumbing-selftest"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=str(ROOT))
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr


def test_watchdog_through_the_spawner():
    # the N>1 watchdog (test_bench_watchdog.py) without torchrun: rank 0's line
    # carries the stuck leg's error and the parent exits with the dog's code
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--watchdog-selftest",
                        "--replica-timeout", "1"], capture_output=True, text=True, timeout=180, env=env,
                       cwd=str(ROOT))
    assert r.returncode == 3, (r.returncode, r.stderr)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["watchdog"]["expired"] is True


def test_ranks_die_with_a_killed_parent():
    """A parent killed outright (SIGKILL at a driver's time limit) leaves no
    rank behind: each child asked for SIGTERM on its parent's death."""
    import signal
    import time

    import psutil
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.Popen([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--watchdog-selftest",
                          "--replica-timeout", "120"], env=env, cwd=str(ROOT),
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        kids = []
        for _ in range(100):                       # both ranks started
            kids = psutil.Process(p.pid).children()
            if len(kids) == 2:
                break
            time.sleep(0.1)
        assert len(kids) == 2
        time.sleep(2.0)                            # let them reach the stuck exchange
        os.kill(p.pid, signal.SIGKILL)
        p.wait(timeout=30)
        gone, alive = psutil.wait_procs(kids, timeout=30)
        assert not alive, [k.pid for k in alive]
    finally:
        if p.poll() is None:
            p.kill()
