"""bench.py --gpus N without a launcher starts the N ranks itself (bench.spawn_ranks): every
rank gets the torch.distributed.run environment, rank 0's stdout is the command's, and a
failing rank fails the command.  CPU only: the workers here are a probe script that joins a
gloo group and reports what it saw, instead of the GPU bench."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r'''
import json, os, sys
import torch.distributed as dist
dist.init_process_group("gloo")
seen = [None] * dist.get_world_size()
dist.all_gather_object(seen, {k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")})
if dist.get_rank() == 0:
    print(json.dumps({"argv": sys.argv[1:], "seen": seen}))
fail = os.environ.get("PROBE_FAIL_RANK")
dist.barrier()
dist.destroy_process_group()
if fail is not None and int(fail) == int(os.environ["RANK"]):
    sys.exit(3)
'''


def _run(tmp_path, n, env_extra=None):
    probe = tmp_path / "probe.py"
    probe.write_text(PROBE)
    code = "import sys; sys.path.insert(0, %r); import bench; sys.exit(bench.spawn_ranks(%d, ['--steps', '4'], script=%r))" % (
        ROOT, n, str(probe))
    env = dict(os.environ, **(env_extra or {}))
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env)


def test_spawn_ranks_environment(tmp_path):
    r = _run(tmp_path, 3)
    assert r.returncode == 0, r.stderr
    # (gloo's own banner goes to stdout too; bench.py itself points fd 1 at stderr)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout      # one JSON line: rank 0's
    out = json.loads(lines[0])
    assert out["argv"] == ["--steps", "4"]
    assert [s["RANK"] for s in out["seen"]] == ["0", "1", "2"]
    assert [s["LOCAL_RANK"] for s in out["seen"]] == ["0", "1", "2"]
    assert all(s["WORLD_SIZE"] == "3" and s["MASTER_ADDR"] == "127.0.0.1" for s in out["seen"])


def test_spawn_ranks_failure_propagates(tmp_path):
    r = _run(tmp_path, 2, {"PROBE_FAIL_RANK": "1"})
    assert r.returncode == 3, (r.returncode, r.stderr)


def test_gpus_flag_must_match_launcher():
    """Under a launcher WORLD_SIZE wins; a --gpus that disagrees is refused before any GPU work."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
