"""Pipelined execution of K steps: the multi-stream schedule issued by the
native launch list (csrc/sched.hip) or eagerly from Python.

The reference's per-frame chain is synchronous (main_preview.py:94-109:
``pipeline(raw) -> detector.infer(proc) -> tracker.update(dets, ts, proj)``).
On the device the three stages of consecutive steps are independent except
through SORT's per-stream state, so a run of K steps is software-pipelined
over four HIP streams.  A *unit* is P consecutive steps (one YOLO forward
over their P*S frames; P = ``eng.pair`` by default, or a per-unit size list
``units`` whose largest entry is at most ``eng.pair`` -- small units at the
two ends shorten the pipeline's fill and drain); unit u has four stages

    P(u)   preprocess of its P steps into letterbox slot u % 4   (stream sp)
    Y1(u)  first half of its forward on lane u % 2                (stream sy)
    Y2(u)  second half + decode into candidate slot u % 4, then
           that slot's NMS                                       (stream sm)
    T(u)   SORT + result hand-back of each step in order         (stream st)

``sync="stage"`` runs them lock-stepped: stage j issues
Y2(j-1) || P(j+1) || Y1(j) || T(j-2) and joins all four before stage j+1.
``sync="flow"`` drops the joins and chains only the real dependencies with
events: Y1(u) after P(u) and Y2(u-2) (its lane's workspace), Y2(u) after Y1(u)
and T(u-4) (its candidate slot), P(u) after Y1(u-4) (its letterbox slot),
T(u) after Y2(u); and P(u+1) after Y1(u)'s forward part 3 (its stem and
model.2, the VALU-bound start of the forward: the median pass of the next
unit then overlaps the MFMA-bound rest of it).  Both give exactly the
results of K sequential step()
calls: every stream's frames reach SORT in order (all T stages run on one
stream), and no buffer is rewritten before its reader finished.

``mode="native"`` records the schedule once (every stream-ordered library
call and every stream wait becomes a node of an rv_sched launch list) and
``run()`` issues it with one C call; ``mode="eager"`` runs the same Python
stage code on every ``run()``.  Neither uses HIP graph capture
(DESIGN.md §5 "Execution").
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import torch

from . import _lib
from .handback import Record

# name -> (op id, index of the stream argument, {arg index: host bytes})
_OPS = {
    "rv_clahe_median_letterbox_u8": (0, 13, {12: 24}),
    "rv_clahe_median_u8": (1, 11, {}),
    "rv_letterbox_u8": (2, 7, {6: 24}),
    "rv_yolo_forward_part": (3, 10, {}),
    "rv_nms_postprocess": (4, 16, {}),
    "rv_sort_update": (5, 16, {8: 48, 9: 72, 10: 8}),
    "rv_results_handback": (6, 10, {}),
    "rv_untracked_metrics": (7, 10, {4: 72, 5: 8}),
}
_FLOAT = (ctypes.c_float, ctypes.c_double)


def _int_value(v) -> int:
    if v is None:
        return 0
    if isinstance(v, ctypes.c_void_p):
        return int(v.value or 0)
    if isinstance(v, ctypes._SimpleCData):
        return int(v.value)
    return int(v)


def _host_bytes(v, n: int) -> Optional[bytes]:
    if v is None:
        return None
    if isinstance(v, ctypes.Array):
        b = bytes(v)
        if len(b) < n:
            raise ValueError(f"host array of {len(b)} B, expected {n}")
        return b[:n]
    addr = _int_value(v)
    return None if addr == 0 else ctypes.string_at(addr, n)


class Schedule:
    """A native launch list (rv_sched_*).  Inside ``recording()`` every
    recordable library call (``_lib.call`` of a name in _OPS) is appended as
    a node instead of running; ``wait_stream`` appends an event record on
    the source stream and a wait on the destination."""

    def __init__(self):
        h = ctypes.c_void_p()
        _lib.call("rv_sched_create", ctypes.byref(h))
        self.h = h
        self._keep: Dict[int, torch.Tensor] = {}  # tensors whose pointers nodes hold

    def keep(self, t) -> None:
        """Hold `t` until close(): a node recorded its device pointer
        (rvs_amd._lib.ptr calls this while recording)."""
        self._keep[id(t)] = t

    def add(self, name: str, args) -> None:
        op, si, host = _OPS[name]
        argtypes = _lib._SIGS[name][1]
        if len(args) != len(argtypes):
            raise ValueError(f"{name}: {len(args)} arguments, expected {len(argtypes)}")
        iargs, fargs, blob = [], [], bytearray()
        for k, (v, t) in enumerate(zip(args, argtypes)):
            if k == si:
                continue
            if k in host:
                b = _host_bytes(v, host[k])
                if b is None:
                    iargs.append(-1)
                else:
                    iargs.append(len(blob))
                    blob += b
                    blob += bytes((-len(blob)) % 8)  # keep every array 8-B aligned
            elif t in _FLOAT:
                fargs.append(float(v))
            else:
                iargs.append(_int_value(v))
        ia = (ctypes.c_int64 * max(1, len(iargs)))(*iargs)
        fa = (ctypes.c_double * max(1, len(fargs)))(*fargs)
        hb = (ctypes.c_uint8 * max(1, len(blob))).from_buffer_copy(bytes(blob) or b"\0")
        _lib.call("rv_sched_add_op", self.h, op, ia, len(iargs), fa, len(fargs), hb, len(blob),
                  _int_value(args[si]))

    def record(self, stream, timing: bool = False) -> int:
        e = ctypes.c_int(-1)
        _lib.call("rv_sched_add_record", self.h, int(stream.cuda_stream), 1 if timing else 0,
                  ctypes.byref(e))
        return e.value

    def event_sync(self, event: int) -> None:
        """Block this thread until record node `event` of the last run()."""
        _lib.call("rv_sched_event_sync", self.h, int(event))

    def event_query(self, event: int) -> bool:
        """True once record node `event` of the last run() has completed
        (non-blocking)."""
        st = _lib.call("rv_sched_event_query", self.h, int(event))
        _lib.check(0 if st >= 0 else st, "rv_sched_event_query")
        return st == 1

    def elapsed_ms(self, a: int, b: int) -> float:
        ms = ctypes.c_float()
        _lib.call("rv_sched_event_elapsed", self.h, int(a), int(b), ctypes.byref(ms))
        return float(ms.value)

    def wait(self, stream, event: int) -> None:
        _lib.call("rv_sched_add_wait", self.h, int(stream.cuda_stream), int(event))

    def wait_stream(self, dst, src) -> None:
        self.wait(dst, self.record(src))

    def num_nodes(self) -> int:
        return int(_lib.load().rv_sched_num_nodes(self.h))

    def run(self, origin=None) -> None:
        o = origin if origin is not None else torch.cuda.current_stream()
        _lib.call("rv_sched_run", self.h, int(o.cuda_stream))

    def recording(self):
        return _lib.recording(self)

    def close(self) -> None:
        if self.h:
            _lib.load().rv_sched_destroy(self.h)
            self.h = None
        self._keep = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _Events:
    """Event bookkeeping of one issue pass: native (schedule nodes) or eager
    (torch events recorded now)."""

    def __init__(self, sched: Optional[Schedule]):
        self.sched = sched
        self.ev: Dict = {}

    def record(self, key, stream, timing: bool = False):
        if self.sched is not None:
            self.ev[key] = self.sched.record(stream, timing)
        else:
            e = torch.cuda.Event(enable_timing=timing)
            e.record(stream)
            self.ev[key] = e

    def wait(self, stream, key):
        if key not in self.ev:
            return
        if self.sched is not None:
            self.sched.wait(stream, self.ev[key])
        else:
            stream.wait_event(self.ev[key])

    def wait_stream(self, dst, src):
        if self.sched is not None:
            self.sched.wait_stream(dst, src)
        else:
            dst.wait_stream(src)


class PipelinedRun:
    """K pipelined steps of a RoadVisionEngine(lanes=2, pair=P) over fixed
    device inputs frames[k] (S,H,W,3) u8 and ts[k] (S,) f64.  After run()
    (and a synchronisation), outs[k] = {"record": step k's pinned host
    record, "proc": step k's proc frames}; the records hold what K step()
    calls would have produced."""

    def __init__(self, eng, frames, ts, mode: str = "native", sync: str = "flow",
                 units: Optional[List[int]] = None):
        if mode not in ("native", "eager"):
            raise ValueError(f"mode {mode!r}: expected 'native' or 'eager'")
        if sync not in ("stage", "flow"):
            raise ValueError(f"sync {sync!r}: expected 'stage' or 'flow'")
        if eng.detector is None:
            raise ValueError("PipelinedRun needs detect.enabled (a detector-off engine runs "
                             "only the preprocess: use step())")
        if eng.detector.lanes != 2:
            raise ValueError("PipelinedRun needs RoadVisionEngine(lanes=2)")
        P = eng.pair
        K = len(frames)
        if units is None:
            if K % P:
                raise ValueError(f"the step count {K} is not a multiple of pair={P}")
            units = [P] * (K // P)
        units = [int(x) for x in units]
        if sum(units) != K or min(units) < 1 or max(units) > P:
            raise ValueError(f"unit sizes {units} must be in [1, pair={P}] and sum to {K}")
        if len(ts) != K:
            raise ValueError("frames and ts differ in length")
        self.eng, self.frames, self.ts = eng, list(frames), list(ts)
        self.mode, self.sync = mode, sync
        self.K, self.P, self.U = K, P, len(units)
        self.units = units
        self.k0 = [sum(units[:u]) for u in range(len(units))]  # first step of unit u
        dev = eng.device
        self.records = [Record(eng.S, eng.detector.max_det, dev) for _ in range(K)]
        # proc outputs: one buffer per step, allocated here (not in the run)
        self.procs = [torch.empty((eng.S, eng.H, eng.W, 3), dtype=torch.uint8, device=dev)
                      for _ in range(K)]
        self.sm, self.sp, self.sy, self.st = (torch.cuda.Stream(dev) for _ in range(4))
        import os
        if os.environ.get("RV_PREP_PRIORITY"):  # A/B probe: the preprocess stream's priority
            self.sp = torch.cuda.Stream(dev, priority=int(os.environ["RV_PREP_PRIORITY"]))
        # A/B probe: RV_HIPRI_STREAMS=sy,sm,st creates those stage streams at
        # high priority (torch: -1), e.g. the later stages ahead of the next
        # units' preprocess during the pipeline fill
        for name in filter(None, os.environ.get("RV_HIPRI_STREAMS", "").split(",")):
            if name not in ("sm", "sp", "sy", "st"):
                raise ValueError(f"RV_HIPRI_STREAMS: unknown stream {name!r}")
            setattr(self, name, torch.cuda.Stream(dev, priority=-1))
        # RV_TRACK_ON_Y2=1: the track stage T(u) runs on the second-half
        # stream right behind Y2(u) (its only producer), one stream fewer
        # competing for the process's hardware queues
        if os.environ.get("RV_TRACK_ON_Y2", "0") != "0":
            self.st = self.sm
        # Y1(u) runs as forward parts 3 + 4 and the preprocess of unit u+1
        # waits for part 3 (the VALU-bound stem and model.2 chain), so the
        # VALU-bound median pass overlaps the MFMA-bound rest of the forward
        # instead of the stem; Y1 is then issued before P (r04: +1.0 % with
        # and without the consumer, five A/B pairs; RV_PREP_AFTER_STEM=0 is
        # the r03 order)
        self.prep_after_stem = os.environ.get("RV_PREP_AFTER_STEM", "1") != "0"
        # unit u's NMS runs on the second-half stream right behind its decode
        # (per-slot NMS outputs), not at the head of T(u): at the end of a
        # run it then overlaps the SORT steps of unit u-1 instead of
        # following them (RV_NMS_ON_Y2=0: the NMS at the head of T(u))
        self.nms_on_y2 = os.environ.get("RV_NMS_ON_Y2", "1") != "0"
        self._nms_out = {}
        self.sched = None
        self._events = None
        if mode == "native":
            self.sched = Schedule()
            with self.sched.recording():
                self._events = _Events(self.sched)
                self._issue(self._events)

    @property
    def outs(self) -> List[dict]:
        return [{"record": r, "proc": p} for r, p in zip(self.records, self.procs)]

    # -- the four stages of unit u ------------------------------------------
    def _prep(self, u: int) -> None:
        eng, S = self.eng, self.eng.S
        slot = u % eng.detector.slots
        for h in range(self.units[u]):
            k = self.k0[u] + h
            eng.preprocess_into(self.frames[k], self.procs[k], slot, h * S)

    def _y1(self, u: int, E: "_Events" = None, stream=None) -> None:
        eng = self.eng
        S, slots = eng.S, eng.detector.slots
        lb = eng.detector.lb[u % slots][:self.units[u] * S]
        if E is None:
            eng.yolo_stage(lb, u % slots, u % 2, part=1)
            return
        eng.yolo_stage(lb, u % slots, u % 2, part=3)
        E.record(("Y1a", u), stream)
        eng.yolo_stage(lb, u % slots, u % 2, part=4)

    def _y2(self, u: int) -> None:
        slots = self.eng.detector.slots
        self.eng.yolo_stage(None, u % slots, u % 2, part=2, batch=self.units[u] * self.eng.S)
        if self.nms_on_y2:
            self._nms_out[u] = self.eng.detector.nms(self.units[u] * self.eng.S, u % slots)

    def _track(self, u: int, E: "_Events") -> None:
        """SORT + hand-back of each step of the unit in order, on the NMS
        output of its slot (run by Y2(u); RV_NMS_ON_Y2=0: here, first); a
        timing event marks each step's completion."""
        eng, S, P = self.eng, self.eng.S, self.units[u]
        if self.nms_on_y2:
            dets, det_n = self._nms_out.pop(u)
        else:
            dets, det_n = eng.detector.nms(S * P, u % eng.detector.slots)
        for h in range(P):
            k = self.k0[u] + h
            eng.track_handback(dets[h * S:(h + 1) * S], det_n[h * S:(h + 1) * S], self.ts[k],
                               self.records[k])
            E.record(("done", k), self.st, timing=True)

    def _issue(self, E: _Events) -> None:
        cur = torch.cuda.current_stream()
        sm, sp, sy, st = self.sm, self.sp, self.sy, self.st
        U, slots = self.U, self.eng.detector.slots
        for x in (sm, sp, sy, st):
            E.wait_stream(x, cur)
        for j in range(-1, U + 2):
            if self.sync == "stage" and j > -1:
                for x in (sp, sy, st):
                    E.wait_stream(x, sm)
            # issue order = the order the HW queues see the stages: Y2, P, Y1, T
            if 0 <= j - 1 < U:  # Y2(j-1): after Y1(j-1), and T(j-1-slots) freed its slot
                u = j - 1
                with torch.cuda.stream(sm):
                    E.wait(sm, ("Y1", u))
                    E.wait(sm, ("T", u - slots))
                    self._y2(u)
                    E.record(("Y2", u), sm)
            if self.prep_after_stem and 0 <= j < U:  # Y1(j) first, as parts 3 + 4
                u = j
                with torch.cuda.stream(sy):
                    E.wait(sy, ("P", u))
                    E.wait(sy, ("Y2", u - 2))
                    self._y1(u, E, sy)
                    E.record(("Y1", u), sy)
            if 0 <= j + 1 < U:  # P(j+1): after Y1(j+1-slots) read its letterbox slot
                u = j + 1
                with torch.cuda.stream(sp):
                    E.wait(sp, ("Y1", u - slots))
                    if self.prep_after_stem:
                        E.wait(sp, ("Y1a", u - 1))
                    self._prep(u)
                    E.record(("P", u), sp)
            if not self.prep_after_stem and 0 <= j < U:  # Y1(j): after P(j), and Y2(j-2) released lane j % 2
                u = j
                with torch.cuda.stream(sy):
                    E.wait(sy, ("P", u))
                    E.wait(sy, ("Y2", u - 2))
                    self._y1(u)
                    E.record(("Y1", u), sy)
            if 0 <= j - 2 < U:  # T(j-2): after Y2(j-2)
                u = j - 2
                with torch.cuda.stream(st):
                    E.wait(st, ("Y2", u))
                    self._track(u, E)
                    E.record(("T", u), st)
            if self.sync == "stage":
                for x in (sp, sy, st):
                    E.wait_stream(sm, x)
        for x in (sm, sp, sy, st):
            E.wait_stream(cur, x)

    def run(self) -> None:
        """Issue the K steps (asynchronous: returns once they are queued)."""
        if self.sched is not None:
            self.sched.run(torch.cuda.current_stream())
        else:
            self._events = _Events(None)
            self._issue(self._events)

    def wait_step(self, k: int) -> None:
        """Block this thread until step k of the last run() has handed its
        results back (its record is then readable)."""
        e = self._events.ev[("done", k)]
        if self.sched is not None:
            self.sched.event_sync(e)
        else:
            e.synchronize()

    def step_ready(self, k: int) -> bool:
        """True once step k of the last run() has handed its results back
        (non-blocking form of wait_step)."""
        e = self._events.ev[("done", k)]
        if self.sched is not None:
            return self.sched.event_query(e)
        return e.query()

    def step_done_ms(self) -> List[float]:
        """Completion time of every step of the last run, in ms after step
        0's (device clock; call after the run has finished)."""
        ev = self._events.ev
        if self.sched is not None:
            return [self.sched.elapsed_ms(ev[("done", 0)], ev[("done", k)]) for k in range(self.K)]
        return [ev[("done", 0)].elapsed_time(ev[("done", k)]) for k in range(self.K)]

    def close(self) -> None:
        if self.sched is not None:
            self.sched.close()
            self.sched = None
