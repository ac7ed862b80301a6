"""CPU: the torch-free process plumbing of the multi-GPU bench and the
sharded align (realsensetracker_amd/rendezvous.py) -- the launcher's rank
environments and the TCP collectives at world size 2 and 3."""
from __future__ import annotations

import multiprocessing as mp
import os
import subprocess
import sys

import numpy as np
import pytest

from realsensetracker_amd import rendezvous as RV


def test_rank_envs():
    envs = RV.rank_envs(4, 29500, base={"PATH": "/bin", "RANK": "9"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_PORT"] == "29500" for e in envs)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" and e["PATH"] == "/bin" for e in envs)
    with pytest.raises(ValueError):
        RV.rank_envs(0, 1)


def _worker(rank, world, port, q):
    r = RV.Rendezvous(rank, world, "127.0.0.1", port, timeout=60)
    r.barrier()
    s = r.allreduce([rank + 1.0, 10.0 * rank], "sum")
    m = r.allreduce([float(rank)], "max")
    b = r.broadcast(b"unique-id-bytes" if rank == 0 else None)
    r.barrier()
    r.close()
    q.put((rank, s.tolist(), float(m[0]), b))


@pytest.mark.parametrize("world", [2, 3])
def test_collectives(world):
    port = RV.free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_sum = [sum(r + 1.0 for r in range(world)), sum(10.0 * r for r in range(world))]
    for rank, s, m, b in out:
        assert s == want_sum and m == world - 1 and b == b"unique-id-bytes"


def test_world_one_needs_no_socket():
    r = RV.Rendezvous(0, 1)
    assert np.array_equal(r.allreduce([2.0, 3.0], "max"), [2.0, 3.0])
    assert r.broadcast(b"x") == b"x"
    r.barrier()


def test_launch_runs_every_rank(tmp_path):
    """bench.py --gpus N without a launcher: N processes with the rank
    environment, the job's status the worst rank's."""
    script = tmp_path / "probe.py"
    root = str(RV.__file__).rsplit("/realsensetracker_amd", 1)[0]
    script.write_text(
        "import os, sys\n"
        f"sys.path.insert(0, {root!r})\n"
        "from realsensetracker_amd import rendezvous as RV\n"
        "w, r, lr = RV.world_from_env()\n"
        "rv = RV.Rendezvous(r, w)\n"
        "tot = rv.allreduce([1.0])[0]\n"
        "open(os.path.join(sys.argv[1], f'rank{r}'), 'w').write(f'{w} {lr} {tot}')\n"
        "rv.close()\n"
        "sys.exit(3 if (r == 1 and len(sys.argv) > 2) else 0)\n")
    code = ("import sys; sys.path.insert(0, %r); from realsensetracker_amd import rendezvous as RV; "
            "sys.exit(RV.launch(int(sys.argv[1]), sys.argv[2:], %r))"
            % (root, str(script)))
    r = subprocess.run([sys.executable, "-c", code, "3", str(tmp_path)], timeout=120)
    assert r.returncode == 0
    for k in range(3):
        assert (tmp_path / f"rank{k}").read_text() == f"3 {k} 3.0"
    r = subprocess.run([sys.executable, "-c", code, "2", str(tmp_path), "fail"], timeout=120)
    assert r.returncode == 3


def test_launch_stops_ranks_when_one_dies_early(tmp_path):
    """A rank that exits non-zero before the collective: the launcher stops
    the ranks blocked in it (they would otherwise wait out the rendezvous
    timeout) and returns the failing rank's status promptly."""
    import time

    script = tmp_path / "early.py"
    root = str(RV.__file__).rsplit("/realsensetracker_amd", 1)[0]
    script.write_text(
        "import sys\n"
        f"sys.path.insert(0, {root!r})\n"
        "from realsensetracker_amd import rendezvous as RV\n"
        "w, r, lr = RV.world_from_env()\n"
        "if r == 2:\n"
        "    sys.exit(5)\n"
        "rv = RV.Rendezvous(r, w, timeout=600)\n"
        "rv.barrier()\n")
    code = ("import sys; sys.path.insert(0, %r); from realsensetracker_amd import rendezvous as RV; "
            "sys.exit(RV.launch(int(sys.argv[1]), sys.argv[2:], %r, grace=2.0))"
            % (root, str(script)))
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code, "3"], timeout=120)
    assert r.returncode == 5
    assert time.monotonic() - t0 < 60


def test_launch_kills_ranks_ignoring_sigterm(tmp_path):
    """Ranks that ignore SIGTERM are killed after the grace period; the job
    timeout reports 124."""
    import time

    script = tmp_path / "stubborn.py"
    script.write_text(
        "import signal, time\n"
        "signal.signal(signal.SIGTERM, signal.SIG_IGN)\n"
        "time.sleep(300)\n")
    root = str(RV.__file__).rsplit("/realsensetracker_amd", 1)[0]
    code = ("import sys; sys.path.insert(0, %r); from realsensetracker_amd import rendezvous as RV; "
            "sys.exit(RV.launch(2, [], %r, grace=1.0, timeout=2.0))" % (root, str(script)))
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], timeout=120)
    assert r.returncode == 124
    assert time.monotonic() - t0 < 30


def test_launch_reports_a_signalled_rank_as_128_plus_n(tmp_path):
    """A rank killed by a signal (Popen's -N) is reported as the shell's
    128 + N, not as sys.exit(-N)'s 256 - N."""
    script = tmp_path / "killed.py"
    script.write_text(
        "import os, signal, sys, time\n"
        "if os.environ['RANK'] == '1':\n"
        "    os.kill(os.getpid(), signal.SIGKILL)\n"
        "time.sleep(300)\n")
    root = str(RV.__file__).rsplit("/realsensetracker_amd", 1)[0]
    code = ("import sys; sys.path.insert(0, %r); from realsensetracker_amd import rendezvous as RV; "
            "sys.exit(RV.launch(2, [], %r, grace=1.0))" % (root, str(script)))
    r = subprocess.run([sys.executable, "-c", code], timeout=120)
    assert r.returncode == 128 + 9


def test_launch_stops_ranks_on_sigterm(tmp_path):
    """SIGTERM to the launcher stops every rank (no orphans) and exits
    128 + 15."""
    import signal
    import time

    script = tmp_path / "sleeper.py"
    script.write_text(
        "import os, sys, time\n"
        "open(sys.argv[1] + '/pid' + os.environ['RANK'], 'w').write(str(os.getpid()))\n"
        "time.sleep(300)\n")
    root = str(RV.__file__).rsplit("/realsensetracker_amd", 1)[0]
    code = ("import sys; sys.path.insert(0, %r); from realsensetracker_amd import rendezvous as RV; "
            "sys.exit(RV.launch(2, [sys.argv[1]], %r, grace=1.0))" % (root, str(script)))
    p = subprocess.Popen([sys.executable, "-c", code, str(tmp_path)])
    t0 = time.monotonic()
    while not all((tmp_path / f"pid{k}").exists() for k in range(2)):
        assert time.monotonic() - t0 < 60
        time.sleep(0.1)
    pids = [int((tmp_path / f"pid{k}").read_text()) for k in range(2)]
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=60) == 128 + 15
    for pid in pids:
        try:
            os.kill(pid, 0)
            alive = True
        except ProcessLookupError:
            alive = False
        assert not alive, pid
