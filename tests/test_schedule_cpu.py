"""Host logic of the native launch list (rvs_amd.schedule / rvs_amd._lib),
no GPU: while a schedule is being recorded, every tensor whose device
pointer a node takes is held by the schedule (a temporary made
during recording was freed while later runs still used its pointer)."""
import gc
import weakref

import torch

from rvs_amd import _lib


class _FakeSchedule:
    def __init__(self):
        self.kept = {}

    def keep(self, t):
        self.kept[id(t)] = t


def test_ptr_keeps_tensors_while_recording():
    rec = _FakeSchedule()
    with _lib.recording(rec):
        t = torch.zeros(16)
        ref = weakref.ref(t)
        p = _lib.ptr(t)
        _lib.ptr(torch.ones(8)[::2].contiguous())  # a temporary, as kernels._frames makes
        del t
        gc.collect()
    assert p != 0 and ref() is not None and len(rec.kept) == 2
    # outside recording nothing is held
    u = torch.zeros(4)
    ref_u = weakref.ref(u)
    _lib.ptr(u)
    del u
    gc.collect()
    assert ref_u() is None and len(rec.kept) == 2
    assert _lib.ptr(None) == 0


def test_schedule_close_releases_kept_tensors():
    from rvs_amd.schedule import Schedule
    s = Schedule.__new__(Schedule)  # no rv_sched_create (it needs the HIP runtime)
    s.h = None
    s._keep = {}
    t = torch.zeros(3)
    ref = weakref.ref(t)
    s.keep(t)
    del t
    gc.collect()
    assert ref() is not None
    s.close()
    gc.collect()
    assert ref() is None
