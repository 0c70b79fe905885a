"""bench.py's multi-rank launch on CPU (gloo): `--gpus N` without a launcher starts N
ranks itself and relays rank 0's line; a world that is not N is refused (VERDICT r2
item 2). `--launch-check` forms the world exactly as the bench does and touches no GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    return env


def _last_json(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


def test_self_launch_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], env=_env(), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2 and line["launch_check"]
    # exactly one line: only rank 0 prints
    assert sum(ln.startswith("{") for ln in r.stdout.splitlines()) == 1


def test_self_launch_bip_workload():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--workload", "bip", "--launch-check"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert _last_json(r.stdout)["n_gpus"] == 2


def test_world_mismatch_is_refused():
    # a rank that finds itself in a 1-rank world while --gpus says 2 must not print a line
    env = _env()
    env.update({"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode != 0
    assert "world that formed" in r.stderr
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())


def test_single_gpu_workload_refuses_many_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--workload", "er-latency", "--launch-check"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "single-GPU" in r.stderr


def test_no_gpu_visible_refuses_before_launch():
    # without --launch-check the parent counts GPUs first: none in this container
    import torch
    if torch.cuda.device_count() >= 2:
        return
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1"], env=_env(), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode != 0 and "GPU(s) visible" in r.stderr
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())


def test_digest_self_check_two_ranks_gloo():
    """the N-rank line's label self-check (replica_digest_checks: MIN
    and MAX all-reduce of every replica's gs_digest, compared with the single-GPU digest)
    over 2 gloo ranks: equal replicas pass, one diverging replica fails both checks."""
    d = "0x8000000000000001"  # above 2^63: the signed all-reduce round trip
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check", "--launch-check-digest", d],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    chk = _last_json(r.stdout)["self_check"]
    assert chk["replica_label_digests_equal"] and chk["digest_equals_single_gpu"]
    assert chk["digest"] == "8000000000000001"
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check", "--launch-check-digest", d,
                        "--launch-check-digest-skew", "7"], env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    chk = _last_json(r.stdout)["self_check"]
    assert not chk["replica_label_digests_equal"] and not chk["digest_equals_single_gpu"]


def test_rccl_channel_knob_reaches_every_rank():
    """--rccl-max-channels sets NCCL_MAX_NCHANNELS before anything initialises
    HIP or RCCL; the self-launched ranks inherit it and report it (config.rccl), checked equal on
    every rank over gloo. Without the flag the line says RCCL's default (None)."""
    env = _env()
    env.pop("NCCL_MAX_NCHANNELS", None)
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check", "--rccl-max-channels", "8"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rc = _last_json(r.stdout)["rccl"]
    assert rc == {"NCCL_MAX_NCHANNELS": 8, "same_on_all_ranks": True}
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert _last_json(r.stdout)["rccl"]["NCCL_MAX_NCHANNELS"] is None
