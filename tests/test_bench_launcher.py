"""bench.py's self-launch for --gpus N > 1 (VERDICT r03 'next' 1) and its watchdog, on the CPU.

The driver may run ``python bench.py --gpus N`` without torch.distributed.run; bench.py then starts the N
ranks itself as one child process (torch.distributed.run, one rank per GPU, RCCL), before anything in the
parent touches a GPU. The dry-run mode prints the child command instead of starting it."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dry_run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args, "--launcher-dry-run"],
                         capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])["launcher"]


def test_launcher_argv_spawns_one_rank_per_gpu():
    j = _dry_run("--gpus", "8", "--steps", "5", "--warmup", "2")
    argv = j["argv"]
    assert j["gpus"] == 8
    assert argv[0] == sys.executable and argv[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in argv and "--nproc-per-node=8" in argv and "--master-addr=127.0.0.1" in argv
    port = [a for a in argv if a.startswith("--master-port=")]
    assert len(port) == 1 and 0 < int(port[0].split("=")[1]) < 65536
    script = argv.index(os.path.join(ROOT, "bench.py"))
    child = argv[script + 1:]
    # the driver's flags are forwarded unchanged; the children skip the one-process line (the parent runs it
    # once the ranks are gone) and rank 0 hands its merged ids to the parent
    assert child[:6] == ["--gpus", "8", "--steps", "5", "--warmup", "2"]
    assert "--launcher-dry-run" not in child
    assert child[child.index("--single-process") + 1] == "0"
    assert child[child.index("--ids-out") + 1].endswith(".npy")


def test_launcher_not_used_under_torchrun_or_single_gpu():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    class A:
        gpus = 2
    argv = bench.launcher_argv(A, ["--gpus", "2", "--launcher-dry-run", "--k", "10"], 29555, "/tmp/x.npy")
    assert argv[argv.index(os.path.join(ROOT, "bench.py")) + 1:][:4] == ["--gpus", "2", "--k", "10"]
    assert "--master-port=29555" in argv


def test_watchdog_reports_a_hang_and_an_error():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    r, e, hung = bench.run_with_watchdog(lambda: time.sleep(3), 0.2)
    assert hung and r is None
    r, e, hung = bench.run_with_watchdog(lambda: 1 / 0, 5)
    assert not hung and isinstance(e, ZeroDivisionError)
    r, e, hung = bench.run_with_watchdog(lambda: 7, 5)
    assert (r, e, hung) == (7, None, False)
    assert bench.EXIT_HUNG != 0


def _bench_module(name):
    import importlib.util

    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


def test_launcher_deadline_kills_a_child_that_hangs_with_stdout_open():
    """the deadline runs from the launch, stdout is read on a helper thread, and the whole process group
    goes when it passes (a rank stuck in a collective keeps torch.distributed.run and its stdout alive)"""
    bench = _bench_module("bench_mod3")
    code = ("import subprocess, sys, time; print('rank output', flush=True); "
            "subprocess.Popen([sys.executable, '-c', 'import time; time.sleep(60)']); time.sleep(60)")
    t0 = time.perf_counter()
    rc, line = bench.run_child([sys.executable, "-c", code], dict(os.environ), 2.0)
    assert rc == 124 and line is None
    assert time.perf_counter() - t0 < 20
    # a child that finishes: its result line comes back, its status too
    code = "import json; print('log'); print(json.dumps({'metric': 'm', 'value': 1}))"
    rc, line = bench.run_child([sys.executable, "-c", code], dict(os.environ), 30.0)
    assert rc == 0 and json.loads(line)["value"] == 1


def test_corpus_modes_weak_and_strong():
    """weak scaling: --rows per rank (configs[3] at N = 8); strong scaling: --rows-total split with the reference's
    'even' rule (gpu_resource_manager.distribute_workload); `value` is full-corpus QPS in both (bench.py docstring)"""
    bench = _bench_module("bench_mod4")

    class A:
        rows, rows_total = 10_000_000, 0
    assert bench.corpus_shards(A, 8) == [(r * 10_000_000, (r + 1) * 10_000_000) for r in range(8)]
    A.rows_total = 10_000_003
    sh = bench.corpus_shards(A, 4)
    assert sh[0] == (0, 2_500_001) and sh[-1][1] == 10_000_003
    assert all(b == a_ for (_, a_), (b, _) in zip(sh[:-1], sh[1:]))
    assert [e - b for b, e in sh] == [2_500_001, 2_500_001, 2_500_001, 2_500_000]
    from gpu_resource_manager import GPUResourceManager, even_split

    assert even_split(10, 3) == [(0, 4), (4, 7), (7, 10)]
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "value = qps_full  # full-corpus QPS" in src and '"shard_searches_per_s"' in src


def test_launcher_forwards_strong_scaling_flags():
    j = _dry_run("--gpus", "4", "--rows-total", "10000000", "--steps", "3")
    child = j["argv"][j["argv"].index(os.path.join(ROOT, "bench.py")) + 1:]
    assert child[:6] == ["--gpus", "4", "--rows-total", "10000000", "--steps", "3"]
