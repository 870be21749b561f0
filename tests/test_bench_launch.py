"""bench.py --gpus N as the driver runs it: without WORLD_SIZE the script is only a launcher that
starts N rank processes with torchrun's environment, never touches torch / libvhx itself, relays a failing rank's
status, and refuses (non-zero, no JSON line) when fewer than N GPUs are visible. CPU only: the ranks of the spawn tests
stop in the VHX_BENCH_RANK_ECHO self-test before importing torch."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "VHX_BENCH_LAUNCHED")}
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True, timeout=300)


def _lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_print_launch_plans_n_ranks_without_torch():
    r = _run(["--gpus", "2", "--print-launch", "--steps", "3"])
    assert r.returncode == 0, r.stderr
    (plan,) = _lines(r.stdout)
    assert plan["world"] == 2 and not plan["torch_imported"] and not plan["vhx_imported"]
    ranks = plan["ranks"]
    assert [p["rank"] for p in ranks] == [0, 1]
    port = ranks[0]["env"]["MASTER_PORT"]
    for p in ranks:
        env = p["env"]
        assert env["RANK"] == env["LOCAL_RANK"] == str(p["rank"])
        assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "2"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == port
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        assert p["cmd"][1] == BENCH and p["cmd"][2:] == ["--gpus", "2", "--steps", "3"]  # no --print-launch


def test_spawns_n_ranks_with_torchrun_environment():
    r = _run(["--gpus", "3", "--steps", "2"], VHX_BENCH_SKIP_DEVICE_CHECK="1", VHX_BENCH_RANK_ECHO="1")
    assert r.returncode == 0, r.stderr
    echoes = sorted((ln["rank_echo"] for ln in _lines(r.stdout)), key=lambda e: int(e["RANK"]))
    assert [e["RANK"] for e in echoes] == ["0", "1", "2"]
    assert all(e["WORLD_SIZE"] == "3" and e["LOCAL_RANK"] == e["RANK"] and e["MASTER_ADDR"] == "127.0.0.1"
               for e in echoes)
    assert len({e["MASTER_PORT"] for e in echoes}) == 1


def test_failing_rank_fails_the_launch():
    r = _run(["--gpus", "2"], VHX_BENCH_SKIP_DEVICE_CHECK="1", VHX_BENCH_RANK_ECHO="fail1")
    assert r.returncode == 3
    assert "rank 1 exited with status 3" in r.stderr


def test_too_few_gpus_refuses_without_a_line():
    # this container has no GPU: two are requested, none are visible
    r = _run(["--gpus", "2"])
    assert r.returncode == 2
    assert "2 GPUs requested" in r.stderr
    assert _lines(r.stdout) == []


def test_gpus_must_match_an_outer_launcher():
    r = _run(["--gpus", "2"], WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "must agree" in r.stderr


@pytest.mark.gpu
def test_gpus_beyond_the_box_refuses_on_gpu():
    """On the one-GPU box: --gpus 2 must fail loudly, never print a one-GPU line."""
    import torch
    n = torch.cuda.device_count()
    r = _run(["--gpus", str(n + 1), "--steps", "1", "--warmup", "0"])
    assert r.returncode == 2, (r.returncode, r.stderr[-500:])
    assert f"{n + 1} GPUs requested, {n} visible" in r.stderr
    assert _lines(r.stdout) == []
