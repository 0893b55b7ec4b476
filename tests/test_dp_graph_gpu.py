"""The DP step captured whole into a HIP graph (bench.py and training.py at N > 1):
forward, backward with parallel.GradReducer's bucketed RCCL all-reduces forked where each bucket is
final (on the capture-only process group, parallel.capture_group), the join and Adam.  Checked on a
1-rank RCCL group in a subprocess (tests/dp_graph_worker.py): graph replays == eager steps bit for bit,
more than one bucket forked during the backward (not all at finish()), a captured collective really
runs on each replay, and eager collectives of the default group right before a capture (the round-4
watchdog abort's precondition) do not disturb it.  The N > 1 arithmetic of the same reducer is
covered over gloo on the CPU (tests/test_parallel.py)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _env():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_hip_rule_event_on_stream_joined_to_capture(gpu):
    """The HIP rule behind the round-4 abort, in isolation: an event recorded eagerly (long complete) on
    a stream that a capture has since joined cannot be queried (hipErrorCapturedEvent, the watchdog's
    error, and the failed query invalidates the capture); the same event can be while a capture that
    its stream did not join runs, and again after the capture ends."""
    r = subprocess.run([sys.executable, os.path.join(HERE, "hip_event_rule_worker.py")], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["eager_before"] == {"done": True}, out
    assert out["capture_not_joined"] == {"done": True}, out
    # exactly the watchdog's error in r04i_pytest_gpu_watchdog_abort.log; the query also invalidates the
    # capture (the next captured operation fails)
    assert "event last recorded in a capturing stream" in out["S_joined"].get("error", ""), out
    assert "previous error during capture" in out["capture_after_query"], out
    assert out["after_capture"] == {"done": True}, out


@pytest.mark.parametrize("name,B,precision", [("mfcc_bgru", 64, "fp32"), ("mfcc_bgru", 64, "bf16")])
def test_dp_step_graph_with_captured_allreduce(gpu, name, B, precision):
    r = subprocess.run([sys.executable, os.path.join(HERE, "dp_graph_worker.py"), name, str(B), precision],
                       env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["buckets"] > 2, out
    assert out["forked_during_backward"] >= 1, out      # overlapped, not all launched at finish()
    assert out["losses_equal"] and out["params_equal"], out
    assert out["spin_timeouts"] == 0, out
    assert out["captured_collective_replays"] == [True, True, True], out
    assert out["eager_then_capture"] == [float(v) for v in range(2, 10)], out


def test_dp_step_graph_flat_allreduce_and_syncbn(gpu):
    """the single flat all-reduce of --no-overlap and SyncBatchNorm1d's exchanges, captured
    right after eager warm-up steps on the default group, run on the capture-only group
    (parallel.group_for_now) and the replays equal the eager steps bit for bit."""
    r = subprocess.run([sys.executable, os.path.join(HERE, "dp_graph_worker.py"), "resnet_bgru", "16", "fp32",
                        "flat_syncbn"], env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    # 1 flat all-reduce + SyncBN statistics for every BatchNorm layer, all on the capture group
    assert len(out["captured_on_capture_group"]) > 10 and all(out["captured_on_capture_group"]), out
    assert out["losses_equal"] and out["params_equal"], out
    assert out["spin_timeouts"] == 0, out
