"""The selection logic of tools/placement.py resident_frames (bench-only)
on the CPU (torch.cuda calls stubbed; a fake operator whose launches on the
second candidate take longer, or shorter): the candidates are timed
alternately, candidate 0 (the plain allocation) is kept unless candidate 1 is
faster by more than the threshold, the kept one holds the fill, both timings
and the margin are reported, the timer is left reset, and the plain paths
(probe=False, no room for two, an empty batch) allocate once."""
import pytest
import torch

from tools import placement


class _FakeOp:
    def __init__(self, slow_second, slow=21.2, fast=20.7):
        self.slow_second = slow_second
        self.slow, self.fast = slow, fast
        self.seen = []
        self.order = []
        self.ms = 0.0
        self.n = 0

    def run_device(self, frames, series, ref=None):
        if frames.data_ptr() not in self.seen:
            self.seen.append(frames.data_ptr())
        idx = self.seen.index(frames.data_ptr())
        self.order.append(idx)
        second = idx == 1
        self.ms += (self.slow if second == self.slow_second else self.fast)
        self.n += 1

    def kernel_time(self, reset=False):
        out = (self.ms, self.n)
        if reset:
            self.ms, self.n = 0.0, 0
        return out


@pytest.fixture
def no_cuda(monkeypatch):
    state = {"free": 1 << 40}
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None: (state["free"], 1 << 40))
    monkeypatch.setattr(torch.cuda, "synchronize", lambda dev=None: None)
    monkeypatch.setattr(torch.cuda, "empty_cache", lambda: None)
    return state


@pytest.mark.parametrize("slow_second", [True, False])
def test_keeps_the_faster_candidate(no_cuda, slow_second):
    op = _FakeOp(slow_second)
    fills = []

    def fill(t):
        t.fill_(7)
        fills.append(t.data_ptr())

    t, rep = placement.resident_frames(op, (4, 3, 5, 3), "cpu", fill, rounds=3)
    assert rep["probe"] and rep["launches_each"] == 3
    assert rep["kept"] == (0 if slow_second else 1)
    assert rep["candidate_kernel_ms"] == ([20.7, 21.2] if slow_second else [21.2, 20.7])
    assert abs(rep["margin"] - ((20.7 / 21.2 - 1) if slow_second else (21.2 / 20.7 - 1))) < 1e-4
    assert t.data_ptr() == fills[rep["kept"]] and int(t.sum()) == 7 * t.numel()
    assert op.kernel_time() == (0.0, 0)  # left reset
    assert op.order == [0, 1] + [0, 1] * 3  # warm launches, then alternated


def test_keeps_the_plain_allocation_within_the_threshold(no_cuda):
    """Candidate 1 faster by 0.5 % (noise for a power-bound kernel): the
    plain allocation stays."""
    op = _FakeOp(False, slow=20.8, fast=20.7)
    t, rep = placement.resident_frames(op, (4, 3, 5, 3), "cpu", lambda x: x.fill_(3))
    assert rep["kept"] == 0 and 0 < rep["margin"] < rep["threshold"] == 0.01
    assert placement.choose(21.0, 20.7)[0] == 1 and placement.choose(20.7, 21.0)[0] == 0


def test_plain_paths(no_cuda):
    op = _FakeOp(True)
    t, rep = placement.resident_frames(op, (4, 3, 5, 3), "cpu", lambda x: x.fill_(1), probe=False)
    assert rep == {"probe": False, "reason": "disabled"} and op.n == 0 and int(t.sum()) == t.numel()
    no_cuda["free"] = 100  # no room for two candidates
    t, rep = placement.resident_frames(op, (4, 3, 5, 3), "cpu", lambda x: x.fill_(1))
    assert rep == {"probe": False, "reason": "no room for two candidates"} and op.n == 0
    no_cuda["free"] = 1 << 40
    t, rep = placement.resident_frames(op, (0, 3, 5, 3), "cpu", lambda x: None)
    assert rep == {"probe": False, "reason": "empty batch"} and tuple(t.shape) == (0, 3, 5, 3)


def test_second_candidate_not_allocatable(no_cuda, monkeypatch):
    op = _FakeOp(True)
    real_empty = torch.empty
    calls = []

    def empty(*a, **k):
        calls.append(1)
        if len(calls) == 2:
            raise torch.cuda.OutOfMemoryError("no room")
        return real_empty(*a, **k)

    monkeypatch.setattr(torch, "empty", empty)
    t, rep = placement.resident_frames(op, (4, 3, 5, 3), "cpu", lambda x: x.fill_(2))
    assert rep == {"probe": False, "reason": "second candidate not allocatable"}
    assert op.n == 0 and int(t.sum()) == 2 * t.numel()
