"""bench.py's self-spawn path (`python bench.py --gpus N` with no launcher environment): the
parent starts N ranks with torchrun's environment contract, relays rank 0's one JSON line, and
turns any rank's failure or a timeout into a non-zero exit.  CPU only: the ranks here are tiny
stand-in scripts, and bench.py itself on a host without a GPU (its ranks must fail loudly)."""
import io
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (stdlib-only at import time)

ENV_KEYS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def _script(tmp_path, body):
    f = tmp_path / "rank.py"
    f.write_text(textwrap.dedent(body))
    return str(f)


def _run(tmp_path, body, n=3, timeout_s=60.0, argv=()):
    out, err = io.StringIO(), io.StringIO()
    rc = bench.spawn_ranks(n, list(argv), timeout_s, script=_script(tmp_path, body), out=out, err=err)
    return rc, out.getvalue(), err.getvalue()


def test_env_per_rank_and_one_json_line(tmp_path):
    body = f"""
        import json, os, sys
        keys = {ENV_KEYS!r}
        env = {{k: os.environ.get(k) for k in keys}}
        with open(os.path.join({str(tmp_path)!r}, "env%s.json" % env["RANK"]), "w") as fh:
            json.dump(dict(env, argv=sys.argv[1:]), fh)
        print("progress line from rank", env["RANK"])
        if env["RANK"] == "0":
            print(json.dumps({{"metric": "m", "n_gpus": int(env["WORLD_SIZE"])}}))
    """
    rc, out, err = _run(tmp_path, body, n=3, argv=["--gpus", "3", "--steps", "1"])
    assert rc == 0, err
    lines = out.strip().splitlines()
    assert len(lines) == 1 and json.loads(lines[0]) == {"metric": "m", "n_gpus": 3}
    envs = [json.loads((tmp_path / f"env{r}.json").read_text()) for r in range(3)]
    ports = {e["MASTER_PORT"] for e in envs}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for r, e in enumerate(envs):
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == (str(r), str(r), "3", "3")
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["argv"] == ["--gpus", "3", "--steps", "1"]
    assert "progress line from rank 1" in err and "progress line from rank 0" in err  # not on stdout


def test_failing_rank_stops_the_job(tmp_path):
    body = """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(120)  # the other ranks would wait forever in a collective
        print('{"metric": "m"}')
    """
    t0 = time.time()
    rc, out, err = _run(tmp_path, body, n=3)
    assert rc == 3 and out == ""
    assert time.time() - t0 < 60, "the surviving ranks must be terminated, not waited for"
    assert "rank 1 exited with 3" in err


def test_crashing_rank_is_nonzero(tmp_path):
    body = """
        import os, signal, time
        if os.environ["RANK"] == "0":
            os.kill(os.getpid(), signal.SIGABRT)
        time.sleep(120)
    """
    rc, out, _ = _run(tmp_path, body, n=2)
    assert rc == 128 + 6 and out == ""


def test_no_json_line_is_nonzero(tmp_path):
    rc, out, err = _run(tmp_path, "print('no json here')\n", n=2)
    assert rc == 1 and out == "" and "0 JSON lines" in err


def test_timeout(tmp_path):
    rc, out, err = _run(tmp_path, "import time\ntime.sleep(120)\n", n=2, timeout_s=2.0)
    assert rc == 124 and "timeout" in err


def test_bench_gpus2_without_launcher_fails_loudly_without_gpu():
    """bench.py --gpus 2 with no WORLD_SIZE takes the self-spawn path; with no GPU here its ranks
    cannot run and the parent must exit non-zero with no bench line (not hang, not print a line)."""
    env = {k: v for k, v in os.environ.items() if k not in ENV_KEYS}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--spawn-timeout", "240"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert r.stdout.strip() == ""
    assert "spawn_ranks: rank" in r.stderr


def test_terminated_launcher_stops_its_ranks(tmp_path):
    """SIGTERM to the launcher (a driver's time limit) stops every rank, and the launcher exits
    128 + 15; the ranks record their pids so the test can check none survives."""
    body = f"""
        import os, time
        with open(os.path.join({str(tmp_path)!r}, "pid%s" % os.environ["RANK"]), "w") as fh:
            fh.write(str(os.getpid()))
        time.sleep(120)
    """
    script = _script(tmp_path, body)
    runner = tmp_path / "launch.py"
    runner.write_text(textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {REPO!r})
        import bench
        sys.exit(bench.spawn_ranks(3, [], 100.0, script={script!r}))
    """))
    p = subprocess.Popen([sys.executable, str(runner)], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    t0 = time.time()
    while len(list(tmp_path.glob("pid*"))) < 3 and time.time() - t0 < 60:
        time.sleep(0.1)
    pids = [int((tmp_path / f"pid{r}").read_text()) for r in range(3)]
    p.terminate()
    rc = p.wait(timeout=60)
    assert rc == 128 + 15
    time.sleep(0.5)
    def alive(pid):
        try:
            with open(f"/proc/{pid}/status") as fh:
                state = [ln for ln in fh if ln.startswith("State:")][0]
        except (FileNotFoundError, IndexError):
            return False
        return " Z " not in state and "zombie" not in state
    for _ in range(50):
        if not any(alive(pid) for pid in pids):
            break
        time.sleep(0.1)
    assert not any(alive(pid) for pid in pids), "a rank survived its launcher"
