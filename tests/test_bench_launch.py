"""bench.py's multi-GPU launcher (CPU, no GPU touched): `python bench.py --gpus N`
outside torchrun starts N ranks itself, a rank count that differs from --gpus is
refused, and strong scaling is the default (BASELINE configs[3]: the same 1M nodes
sharded over 2/4/8 GPUs)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT")}
    env.update(kw)
    return env


def _last_json(out):
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


def test_self_launch_starts_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-backend", "gloo",
                        "--config", "C3", "--dry-run"], capture_output=True, text=True,
                       timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    out = _last_json(r.stdout)
    assert out["n_gpus"] == 2 and out["rank_sum"] == 1 and out["scaling"] == "strong"
    # the per-rank table of an N > 1 line, gathered over the ranks' group
    ranks = out["ranks"]
    assert set(ranks["per_rank"]) == {"step_ms", "reduce_ms", "fit_ms", "allreduce_ms",
                                      "reduce_frac"}
    assert ranks["per_rank"]["step_ms"] == [1.0, 2.0]
    assert ranks["step_ms_max"] == 2.0 and ranks["step_ms_min"] == 1.0
    assert ranks["allreduce_ms"] == 0.5


def test_rank_count_mismatch_is_refused():
    # a torchrun-style environment with one rank but --gpus 2: no line for the wrong N
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True,
                       text=True, timeout=120,
                       env=_env(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0"))
    assert r.returncode == 2
    assert "refusing" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_single_rank_dry_run():
    r = subprocess.run([sys.executable, BENCH, "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    assert _last_json(r.stdout)["n_gpus"] == 1
