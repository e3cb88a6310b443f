"""bench.py's self-launch: a bare `python bench.py --gpus N` (no WORLD_SIZE) must
start `python -m torch.distributed.run --nproc-per-node N bench.py ...` as a CHILD process before
importing torch, relay rank 0's JSON line to stdout and exit with the child's return code. CPU only:
the real torchrun is exercised with --dry-run (no GPU), the rc/relay rules with stand-in children."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_launch_command_shape():
    cmd = bench.launch_command(["--gpus", "8", "--steps", "5"], 8, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5"]  # the same bench arguments


def test_self_launch_relays_json_and_child_rc(capsys):
    code = "print('rank chatter'); print(json.dumps({'metric': 'm', 'value': 1})); sys.exit(3)"
    rc = bench.self_launch([], 2, cmd=[sys.executable, "-c", "import json, sys; " + code])
    out = capsys.readouterr()
    assert rc == 3  # the child's failure propagates
    assert json.loads(out.out.strip()) == {"metric": "m", "value": 1}  # only the JSON line on stdout
    assert "rank chatter" in out.err


def test_self_launch_no_json_is_a_failure(capsys):
    assert bench.self_launch([], 2, cmd=[sys.executable, "-c", "print('nothing')"]) == 1
    assert bench.self_launch([], 2, cmd=[sys.executable, "-c", "import sys; sys.exit(5)"]) == 5


def test_bare_bench_starts_n_ranks_through_torchrun():
    # the real path: bench.py --gpus 2 (no WORLD_SIZE) -> torchrun child -> 2 ranks; rank 0's line relayed
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["gpus_arg"] == 2 and rec["master_addr"] == "127.0.0.1"
    assert rec["argv"] == ["--gpus", "2", "--dry-run", "--steps", "3"]


def test_bare_bench_propagates_a_failing_rank():
    # without a GPU the ranks fail in torch.cuda.set_device: the parent must exit non-zero, no JSON
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=dict(_env(), CUDA_VISIBLE_DEVICES=""),
                       cwd=ROOT)
    assert r.returncode != 0
    assert r.stdout.strip() == ""


def test_self_launch_budget_kills_the_ranks_and_reports_their_phase(capsys, tmp_path):
    # a rank stuck (here: asleep) must not hold the launch past its budget; the whole
    # process group goes, the parent returns 124 and prints where each rank stopped
    import time
    child = ("import os, time; d = os.environ['DFAMD_PROGRESS_DIR']; "
             "open(os.path.join(d, 'rank0.log'), 'a').write('00:00:00 0.0 c4: timed (50 calls)\\n'); "
             "open(os.path.join(d, 'rank1.log'), 'a').write('00:00:00 0.0 c4: create (df_create, step 0)\\n'); "
             "time.sleep(120)")
    env_before = os.environ.pop(bench.PROGRESS_ENV, None)
    t0 = time.monotonic()
    try:
        rc = bench.self_launch([], 2, cmd=[sys.executable, "-c", child], timeout_s=3)
    finally:
        if env_before is not None:
            os.environ[bench.PROGRESS_ENV] = env_before
    took = time.monotonic() - t0
    err = capsys.readouterr().err
    assert rc == 124
    assert took < 30, took
    assert "budget of 3 s exceeded" in err
    assert "rank0: last phase 'c4: timed (50 calls)'" in err
    assert "rank1: last phase 'c4: create (df_create, step 0)'" in err


def test_bare_bench_ranks_record_their_phases(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=dict(_env(), DFAMD_PROGRESS_DIR=str(tmp_path)),
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    for rank in (0, 1):
        lines = (tmp_path / f"rank{rank}.log").read_text().splitlines()
        assert lines and lines[-1].endswith("dry-run"), lines


def test_signal_to_the_launcher_ends_the_ranks(tmp_path):
    # the ranks run in their own session; a SIGTERM to the launcher (an outer `timeout`) must end
    # their process group too, not leave them holding the GPUs
    import signal
    import time
    pidf = tmp_path / "child.pid"
    child = f"import os, time; open({str(pidf)!r}, 'w').write(str(os.getpid())); time.sleep(120)"
    launcher = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
                f"sys.exit(bench.self_launch([], 2, cmd=[sys.executable, '-c', {child!r}], timeout_s=600))")
    p = subprocess.Popen([sys.executable, "-c", launcher], env=_env(), stderr=subprocess.PIPE, text=True)
    t0 = time.monotonic()
    while not pidf.exists() or not pidf.read_text():
        assert time.monotonic() - t0 < 60 and p.poll() is None
        time.sleep(0.1)
    cpid = int(pidf.read_text())
    p.send_signal(signal.SIGTERM)
    rc = p.wait(60)
    err = p.stderr.read()
    assert rc == 128 + signal.SIGTERM, (rc, err[-2000:])
    assert "terminating the ranks" in err
    for _ in range(100):  # the child is gone (reaped by the launcher before it exited)
        try:
            os.kill(cpid, 0)
        except ProcessLookupError:
            break
        time.sleep(0.1)
    else:
        os.kill(cpid, signal.SIGKILL)
        raise AssertionError("the rank outlived its launcher")
