"""bench.py's own rank launcher (krcn.launch), on CPU with the gloo backend.

`python bench.py --gpus N` outside torchrun starts N rank processes with the
torchrun environment; here the same launcher runs a gloo all-reduce at world
size 2, a failing rank must fail the whole launch, and bench.py must refuse a
request for more GPUs than are visible (this container has none) instead of
reporting a smaller run.
"""
import os
import subprocess
import sys
import textwrap
import time

from krcn import launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "krylov-cubic-regularized-newton_amd")

_RANK_SCRIPT = textwrap.dedent("""
    import os, sys
    import torch, torch.distributed as dist
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    assert int(os.environ["LOCAL_RANK"]) == r and os.environ["MASTER_ADDR"] == "127.0.0.1"
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    if r == 0:
        open(sys.argv[1], "w").write(f"{w} {t.item()}")
    dist.destroy_process_group()
""")


def test_launch_two_gloo_ranks(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    out = tmp_path / "out.txt"
    rc = launch.launch_ranks(2, [str(script), str(out)])
    assert rc == 0
    assert out.read_text() == "2 3.0"


def test_failing_rank_fails_the_launch(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "sys.exit(3) if os.environ['RANK'] == '1' else time.sleep(60)\n")
    t0 = time.time()
    rc = launch.launch_ranks(2, [str(script)])
    assert rc == 3
    assert time.time() - t0 < 30   # the surviving rank was terminated, not waited for


def _bench(args, env_extra=None):
    env = dict(os.environ)
    for k in launch.ENV_KEYS:
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=300)


def test_bench_refuses_more_gpus_than_visible():
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "requested but only" in r.stderr
    assert '"metric"' not in r.stdout


def test_bench_refuses_world_mismatch():
    r = _bench(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_hung_ranks_time_out(tmp_path):
    """A rank stuck in a collective never exits: the launcher's timeout ends
    every rank and reports 124 instead of waiting forever."""
    script = tmp_path / "rank.py"
    script.write_text("import time\ntime.sleep(120)\n")
    t0 = time.time()
    rc = launch.launch_ranks(2, [str(script)], timeout=2)
    assert rc == 124
    assert time.time() - t0 < 30
