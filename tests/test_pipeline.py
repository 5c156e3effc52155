"""PipelinedBatchRunner's host logic (bench.py's in-flight steps) with stand-in runners:
every step runs exactly once, on one slot, into its own result buffer, and the results are
read back from the slot that ran it; an error in a slot's call reaches the caller."""
import os
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "se3-icp_amd"))

from se3icp.registration import PipelinedBatchRunner  # noqa: E402


class _Stub:
    def __init__(self, slot, log, fail_at=None):
        self.slot, self.log, self.fail_at = slot, log, fail_at
        self.buf = {}

    def run(self, i):
        if self.fail_at is not None and i == self.fail_at:
            raise RuntimeError(f"slot {self.slot} step {i}")
        time.sleep(0.002 * (1 + self.slot))
        self.log.append((self.slot, i, threading.get_ident()))
        self.buf[i] = ("result", self.slot, i)

    def results(self, i):
        return self.buf[i]

    def kernel_times(self, i):
        return {"slot": self.slot, "step": i}


@pytest.mark.parametrize("in_flight,steps", [(1, 5), (2, 1), (2, 7), (3, 10)])
def test_every_step_once_on_its_owner(in_flight, steps):
    log = []
    pipe = PipelinedBatchRunner(lambda k: _Stub(k, log), in_flight=in_flight, steps=steps)
    pipe.run_steps()
    ran = sorted(i for _, i, _ in log)
    assert ran == list(range(steps))
    for s in range(steps):
        k = pipe.owner(s)
        assert 0 <= k < in_flight
        assert pipe.results(s) == ("result", k, s)
        assert pipe.kernel_times(s) == {"slot": k, "step": s}
    if in_flight > 1 and steps >= in_flight:
        assert len({t for _, _, t in log}) > 1  # (the slots ran from their own threads)


def test_warm_runs_each_slot_once():
    log = []
    pipe = PipelinedBatchRunner(lambda k: _Stub(k, log), in_flight=2, steps=3)
    pipe.warm()
    assert sorted((k, i) for k, i, _ in log) == [(0, 0), (1, 0)]


def test_error_in_a_slot_reaches_the_caller():
    log = []
    pipe = PipelinedBatchRunner(lambda k: _Stub(k, log, fail_at=3), in_flight=2, steps=6)
    with pytest.raises(RuntimeError):
        pipe.run_steps()
