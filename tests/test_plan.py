"""Launch plans (csrc/runtime/plan.h) on the host: recording, replay order of Python ops,
nesting errors and abort.  Kernel launches inside plans are covered on the GPU
(test_executor_gpu.py::test_launch_plan_matches_eager, test_ddp_gpu.py)."""
import pytest

import pgdist  # noqa: F401
from pgdist.ops import kernels as K


def test_plan_records_and_replays_python_ops_in_order():
    log = []
    plan = K.LaunchPlan()

    def step():
        K.plan_py(lambda: log.append("a"))
        log.append("not-recorded")
        K.plan_py(lambda: log.append("b"))

    plan.record(step)
    assert log == ["a", "not-recorded", "b"]
    assert len(plan) == 2
    log.clear()
    plan.replay()
    plan.replay()
    assert log == ["a", "b", "a", "b"]
    plan.free()
    assert len(plan) == 0


def test_plan_nested_recording_rejected_and_abort():
    plan = K.LaunchPlan()

    def bad():
        K.plan_py(lambda: None)
        raise KeyError("boom")

    with pytest.raises(KeyError):
        plan.record(bad)
    assert not K.plan_recording()          # aborted: a new recording can start
    inner = K.LaunchPlan()

    def nested():
        inner.record(lambda: None)

    with pytest.raises(RuntimeError, match="already open"):
        plan.record(nested)
    assert not K.plan_recording()


def test_plan_py_outside_recording_just_runs():
    hits = []
    K.plan_py(lambda: hits.append(1))
    assert hits == [1]
