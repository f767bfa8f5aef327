"""CPU: bench.py keeps the driver's contract without running it (that needs a
GPU): the metric is BASELINE.json's, the defaults are one GPU and a bounded
run at config 3, and the CPU-baseline leg (the test-only oracle) reports the
fields the bench line carries."""
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    return importlib.import_module("bench")  # the repo root is on sys.path (conftest.py)


def test_metric_is_baselines():
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert _bench().METRIC == base["metric"]


def test_defaults_are_one_gpu_config3(monkeypatch):
    b = _bench()
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = b.parse()
    assert (a.gpus, a.envs_per_gpu, a.precision) == (1, 262_144, "f32")
    assert a.steps > 0 and a.warmup >= 0 and a.graph_steps > 0 and not a.no_obs
    assert a.dist_backend == "nccl"


def test_cpu_baseline_fields():
    b = _bench()
    r = b.cpu_baseline(0.3, 2, 0)
    assert set(r) >= {"value", "unit", "cores", "kind", "sample"}
    assert r["kind"] == "port" and r["cores"] == 2 and r["value"] > 0
