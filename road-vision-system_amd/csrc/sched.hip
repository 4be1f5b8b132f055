// Native launch schedule: the multi-stream pipeline of K steps, recorded once
// and issued by one call per run (rvs_amd/schedule.py builds it).
//
// The reference runs its per-frame chain synchronously, one call after the
// other (main_preview.py:94-109: pipeline -> detector.infer -> tracker.update).
// Here a run of K steps is a list of nodes, each either one stream-ordered
// C-ABI call of this library with its arguments frozen at record time (the
// fused preprocess, a forward half, NMS, SORT, the result hand-back), an
// event record on a stream, or a stream's wait on such an event.  rv_sched_run
// forks every stream of the schedule from the caller's stream, issues the
// nodes in record order and joins them back, so the caller's stream sees the
// whole run as one stream-ordered operation.
//
// Why not HIP graphs: multi-stream stream capture and replay of the same
// schedule segfaulted intermittently inside the ROCm runtime (host side:
// hipStreamEndCapture / hipGraphLaunch; DESIGN.md §5 "Execution").  The
// launches here are ordinary stream launches -- the most exercised path of
// the runtime -- and the host cost is one C call per run plus a few
// microseconds per launch, far below the device time of a step.
//
// Host-array arguments (the letterbox geometry, SORT's parameter block and
// homography) are copied into the node at record time.
#include <atomic>
#include <vector>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "common.h"

namespace rv {
namespace {

enum NodeKind { kOp = 0, kRecord = 1, kWait = 2 };

struct Node {
  int kind = kOp;
  int op = 0;
  hipStream_t st = nullptr;
  int event = -1;
  std::vector<int64_t> i;     // integer / pointer / size arguments, in order
  std::vector<double> f;      // float / double arguments, in order
  std::vector<uint8_t> host;  // host arrays; an i-slot holds its offset (or -1)
};

struct Schedule {
  std::vector<Node> nodes;
  std::vector<hipEvent_t> events;
  std::vector<hipStream_t> streams;  // every stream a node runs on (fork / join set)
  hipEvent_t fork = nullptr;
  std::vector<hipEvent_t> join;
  int64_t runs = 0;
  // run generations: a run stamps every record node it issues with its
  // generation; done_gen is the generation of the latest run that issued all
  // its nodes (-1 while a run is issuing or after a failed one).  A host wait
  // is valid only on an event of run done_gen.
  std::vector<int64_t> ev_gen;
  std::atomic<int64_t> gen{0};
  std::atomic<int64_t> done_gen{-1};
};

template <class T>
T* P(int64_t v) {
  return reinterpret_cast<T*>(static_cast<intptr_t>(v));
}

const void* host_arg(const Node& n, int64_t off) {
  return off < 0 ? nullptr : n.host.data() + off;
}

// The recordable calls.  Argument order = the C signature in include/rvhip.h
// with float-class arguments moved to `f` (their relative order kept).
struct OpSpec {
  int ni, nf;
};
const OpSpec kSpecs[RV_SCHED_NUM_OPS] = {
    /* RV_SCHED_CLAHE_MEDIAN_LETTERBOX */ {12, 1},
    /* RV_SCHED_CLAHE_MEDIAN */ {10, 1},
    /* RV_SCHED_LETTERBOX */ {7, 0},
    /* RV_SCHED_YOLO_FORWARD_PART */ {10, 1},
    /* RV_SCHED_NMS */ {14, 2},
    /* RV_SCHED_SORT_UPDATE */ {16, 0},
    /* RV_SCHED_HANDBACK */ {10, 0},
    /* RV_SCHED_UNTRACKED */ {9, 1},
};

int issue_op(const Node& n) {
  const std::vector<int64_t>& a = n.i;
  const std::vector<double>& f = n.f;
  void* s = n.st;
  switch (n.op) {
    case RV_SCHED_CLAHE_MEDIAN_LETTERBOX:
      // in, out, B, H, W, pitch, tiles, [clip], k, ws, ws_bytes, lb_out, geo(host)
      return rv_clahe_median_letterbox_u8(P<const uint8_t>(a[0]), P<uint8_t>(a[1]), (int)a[2],
                                          (int)a[3], (int)a[4], (int)a[5], (int)a[6], f[0],
                                          (int)a[7], P<void>(a[8]), (size_t)a[9],
                                          P<uint8_t>(a[10]), (const int*)host_arg(n, a[11]), s);
    case RV_SCHED_CLAHE_MEDIAN:
      // in, out, B, H, W, pitch, tiles, [clip], k, ws, ws_bytes
      return rv_clahe_median_u8(P<const uint8_t>(a[0]), P<uint8_t>(a[1]), (int)a[2], (int)a[3],
                                (int)a[4], (int)a[5], (int)a[6], f[0], (int)a[7], P<void>(a[8]),
                                (size_t)a[9], s);
    case RV_SCHED_LETTERBOX:
      // in, out, B, H, W, pitch, geo(host)
      return rv_letterbox_u8(P<const uint8_t>(a[0]), P<uint8_t>(a[1]), (int)a[2], (int)a[3],
                             (int)a[4], (int)a[5], (const int*)host_arg(n, a[6]), s);
    case RV_SCHED_YOLO_FORWARD_PART:
      // handle, lb, B, ws, ws_bytes, raw, [conf], cand, cap, seg_n, part
      return rv_yolo_forward_part(P<void>(a[0]), P<const uint8_t>(a[1]), (int)a[2], P<void>(a[3]),
                                  (size_t)a[4], P<float>(a[5]), (float)f[0], P<void>(a[6]),
                                  (int)a[7], P<int>(a[8]), s, (int)a[9]);
    case RV_SCHED_NMS:
      // cand, seg_n, B, cap, nseg, [iou], max_det, max_nms, [max_wh], scale5, keep, out,
      // out_n, cand_total, ws, ws_bytes
      return rv_nms_postprocess(P<const void>(a[0]), P<const int>(a[1]), (int)a[2], (int)a[3],
                                (int)a[4], (float)f[0], (int)a[5], (int)a[6], (float)f[1],
                                P<const float>(a[7]), P<const uint32_t>(a[8]), P<float>(a[9]),
                                P<int>(a[10]), P<int>(a[11]), P<void>(a[12]), (size_t)a[13], s);
    case RV_SCHED_SORT_UPDATE:
      // state_in, state_out, S, tmax, dets, dcount, dmax, ts, params6(host), H9(host),
      // origin2(host), ws, ws_bytes, out_id, out_dist, out_speed
      return rv_sort_update(P<void>(a[0]), P<void>(a[1]), (int)a[2], (int)a[3],
                            P<const float>(a[4]), P<const int>(a[5]), (int)a[6],
                            P<const double>(a[7]), (const double*)host_arg(n, a[8]),
                            (const double*)host_arg(n, a[9]), (const float*)host_arg(n, a[10]),
                            P<void>(a[11]), (size_t)a[12], P<int>(a[13]), P<double>(a[14]),
                            P<double>(a[15]), s);
    case RV_SCHED_HANDBACK:
      // dets, det_n, track_id, dist, speed, S, dmax, stage, stage_bytes, host_dst
      return rv_results_handback(P<const float>(a[0]), P<const int>(a[1]), P<const int>(a[2]),
                                 P<const double>(a[3]), P<const double>(a[4]), (int)a[5],
                                 (int)a[6], P<void>(a[7]), (size_t)a[8], P<void>(a[9]), s);
    case RV_SCHED_UNTRACKED:
      // dets, det_n, S, dmax, H9(host), origin2(host), [max_distance], out_id, out_dist,
      // out_speed
      return rv_untracked_metrics(P<const float>(a[0]), P<const int>(a[1]), (int)a[2], (int)a[3],
                                  (const double*)host_arg(n, a[4]),
                                  (const float*)host_arg(n, a[5]), f[0], P<int>(a[6]),
                                  P<double>(a[7]), P<double>(a[8]), s);
  }
  set_error("rv_sched: unknown op %d", n.op);
  return RV_EINVAL;
}

void add_stream(Schedule* S, hipStream_t st) {
  for (hipStream_t x : S->streams)
    if (x == st) return;
  S->streams.push_back(st);
}

void destroy(Schedule* S) {
  for (hipEvent_t e : S->events) (void)hipEventDestroy(e);
  for (hipEvent_t e : S->join) (void)hipEventDestroy(e);
  if (S->fork) (void)hipEventDestroy(S->fork);
  delete S;
}

int new_event(hipEvent_t* e) {
  return hip_check(hipEventCreateWithFlags(e, hipEventDisableTiming), "rv_sched hipEventCreate");
}

}  // namespace
}  // namespace rv

using namespace rv;

extern "C" int rv_sched_create(void** handle) {
  RV_CHECK_ARG(handle != nullptr, "null handle");
  Schedule* S = new Schedule();
  const int e = new_event(&S->fork);
  if (e) {
    destroy(S);
    *handle = nullptr;
    return e;
  }
  *handle = S;
  return RV_OK;
}

extern "C" int rv_sched_destroy(void* handle) {
  if (handle) destroy(static_cast<Schedule*>(handle));
  return RV_OK;
}

extern "C" int rv_sched_add_op(void* handle, int op, const int64_t* iargs, int ni,
                               const double* fargs, int nf, const void* host, size_t host_bytes,
                               void* stream) {
  RV_CHECK_ARG(handle != nullptr, "null handle");
  RV_CHECK_ARG(op >= 0 && op < RV_SCHED_NUM_OPS, "rv_sched_add_op: unknown op %d", op);
  RV_CHECK_ARG(ni == kSpecs[op].ni && nf == kSpecs[op].nf,
               "rv_sched_add_op(op %d): %d integer / %d float arguments, expected %d / %d", op, ni,
               nf, kSpecs[op].ni, kSpecs[op].nf);
  RV_CHECK_ARG((ni == 0 || iargs) && (nf == 0 || fargs) && (host_bytes == 0 || host),
               "rv_sched_add_op: null argument array");
  Schedule* S = static_cast<Schedule*>(handle);
  Node n;
  n.kind = kOp;
  n.op = op;
  n.st = as_stream(stream);
  n.i.assign(iargs, iargs + ni);
  n.f.assign(fargs, fargs + nf);
  if (host_bytes) n.host.assign((const uint8_t*)host, (const uint8_t*)host + host_bytes);
  S->nodes.push_back(std::move(n));
  add_stream(S, as_stream(stream));
  return RV_OK;
}

extern "C" int rv_sched_add_record(void* handle, void* stream, int timing, int* event) {
  RV_CHECK_ARG(handle != nullptr && event != nullptr, "null pointer");
  Schedule* S = static_cast<Schedule*>(handle);
  hipEvent_t e = nullptr;
  const int st = timing ? hip_check(hipEventCreate(&e), "rv_sched hipEventCreate(timing)")
                        : new_event(&e);
  if (st) return st;
  S->events.push_back(e);
  S->ev_gen.push_back(-1);
  const int id = (int)S->events.size() - 1;
  Node n;
  n.kind = kRecord;
  n.st = as_stream(stream);
  n.event = id;
  S->nodes.push_back(std::move(n));
  add_stream(S, as_stream(stream));
  *event = id;
  return RV_OK;
}

extern "C" int rv_sched_add_wait(void* handle, void* stream, int event) {
  RV_CHECK_ARG(handle != nullptr, "null handle");
  Schedule* S = static_cast<Schedule*>(handle);
  RV_CHECK_ARG(event >= 0 && event < (int)S->events.size(), "rv_sched_add_wait: event %d", event);
  Node n;
  n.kind = kWait;
  n.st = as_stream(stream);
  n.event = event;
  S->nodes.push_back(std::move(n));
  add_stream(S, as_stream(stream));
  return RV_OK;
}

// Host wait for the last run's record node `event` (e.g. one step's result
// hand-back): a consumer thread can take a step's results while later steps
// still run.  Blocks the calling thread only.
extern "C" int rv_sched_event_sync(void* handle, int event) {
  RV_CHECK_ARG(handle != nullptr, "null handle");
  Schedule* S = static_cast<Schedule*>(handle);
  RV_CHECK_ARG(event >= 0 && event < (int)S->events.size(), "rv_sched_event_sync: event %d", event);
  const int64_t g = S->done_gen.load();
  RV_CHECK_ARG(g >= 0 && S->ev_gen[event] == g,
               "rv_sched_event_sync: event %d was not issued by the latest completed run (call it "
               "after rv_sched_run returned without error)", event);
  // poll (default): query + short sleeps, so a waiting consumer never enters
  // the runtime's blocking wait while another thread is still issuing;
  // RV_SCHED_WAIT=sync: hipEventSynchronize
  static const bool use_sync = getenv("RV_SCHED_WAIT") && !strcmp(getenv("RV_SCHED_WAIT"), "sync");
  if (use_sync)
    return hip_check(hipEventSynchronize(S->events[event]), "rv_sched hipEventSynchronize");
  for (;;) {
    const hipError_t e = hipEventQuery(S->events[event]);
    if (e == hipSuccess) return RV_OK;
    if (e != hipErrorNotReady) return hip_check(e, "rv_sched hipEventQuery");
    usleep(50);
  }
}

// Non-blocking: 1 if the last run's record node `event` has completed, 0 if
// not yet (same validity rule as rv_sched_event_sync), so a consumer can do
// other work -- e.g. prepare the objects it will fill -- while it waits.
extern "C" int rv_sched_event_query(void* handle, int event) {
  RV_CHECK_ARG(handle != nullptr, "null handle");
  Schedule* S = static_cast<Schedule*>(handle);
  RV_CHECK_ARG(event >= 0 && event < (int)S->events.size(), "rv_sched_event_query: event %d", event);
  const int64_t g = S->done_gen.load();
  RV_CHECK_ARG(g >= 0 && S->ev_gen[event] == g,
               "rv_sched_event_query: event %d was not issued by the latest completed run", event);
  const hipError_t e = hipEventQuery(S->events[event]);
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) return 0;
  return hip_check(e, "rv_sched hipEventQuery");
}

// Milliseconds between two timing record nodes of the last run.
extern "C" int rv_sched_event_elapsed(void* handle, int a, int b, float* ms) {
  RV_CHECK_ARG(handle != nullptr && ms != nullptr, "null pointer");
  Schedule* S = static_cast<Schedule*>(handle);
  const int n = (int)S->events.size();
  RV_CHECK_ARG(a >= 0 && a < n && b >= 0 && b < n, "rv_sched_event_elapsed: events %d %d", a, b);
  const int64_t g = S->done_gen.load();
  RV_CHECK_ARG(g >= 0 && S->ev_gen[a] == g && S->ev_gen[b] == g,
               "rv_sched_event_elapsed: events %d %d were not issued by the latest completed run", a, b);
  return hip_check(hipEventElapsedTime(ms, S->events[a], S->events[b]),
                   "rv_sched hipEventElapsedTime");
}

extern "C" int rv_sched_num_nodes(void* handle) {
  return handle ? (int)static_cast<Schedule*>(handle)->nodes.size() : 0;
}

extern "C" int rv_sched_run(void* handle, void* origin) {
  RV_CHECK_ARG(handle != nullptr, "null handle");
  Schedule* S = static_cast<Schedule*>(handle);
  hipStream_t o = as_stream(origin);
  while (S->join.size() < S->streams.size()) {
    hipEvent_t e = nullptr;
    const int st = new_event(&e);
    if (st) return st;
    S->join.push_back(e);
  }
  S->done_gen.store(-1);
  const int64_t gen = S->gen.fetch_add(1) + 1;
  int st = hip_check(hipEventRecord(S->fork, o), "rv_sched fork record");
  for (hipStream_t x : S->streams)
    if (!st && x != o) st = hip_check(hipStreamWaitEvent(x, S->fork, 0), "rv_sched fork wait");
  for (size_t k = 0; k < S->nodes.size() && !st; ++k) {
    const Node& n = S->nodes[k];
    if (n.kind == kOp) {
      st = issue_op(n);
    } else if (n.kind == kRecord) {
      st = hip_check(hipEventRecord(S->events[n.event], n.st), "rv_sched hipEventRecord");
      if (!st) S->ev_gen[n.event] = gen;
    } else {
      st = hip_check(hipStreamWaitEvent(n.st, S->events[n.event], 0), "rv_sched hipStreamWaitEvent");
    }
  }
  // join every stream back into the origin, also after a failed node (so the
  // caller's stream never runs ahead of work already queued)
  for (size_t k = 0; k < S->streams.size(); ++k) {
    hipStream_t x = S->streams[k];
    if (x == o) continue;
    int e = hip_check(hipEventRecord(S->join[k], x), "rv_sched join record");
    if (!e) e = hip_check(hipStreamWaitEvent(o, S->join[k], 0), "rv_sched join wait");
    if (!st) st = e;
  }
  if (!st) {
    S->runs++;
    S->done_gen.store(gen);
  }
  return st;
}
