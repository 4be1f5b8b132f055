// Frame capture front end (the reference's VideoSource,
// src/io_video/capture.py:10-24, and README module 8's async pipeline).
//
// Host code: one reader thread per source reads frames from a file into a
// ring of pinned host slots (hipHostMalloc; pageable when no HIP device is
// present, e.g. the CPU test container), stamping each with the wall-clock
// time it was read (capture.py:20: ts = time.time() after cap.read()).  The
// consumer takes filled slots in order and hands them back when done.
//
// rv_capture_upload_batch feeds RoadVisionEngine: for S sources it takes one
// frame of each, queues its H2D copy on the caller's stream and records an
// event behind it; the slot returns to its reader once that event has
// completed (polled at the next upload; waited for -- the oldest copy only --
// when the next slot in order is still held by an earlier upload) -- so the
// ring refills while the device works
// and nothing blocks on a copy in flight.  No host callbacks are queued in
// streams.  Frames travel as NV12 (1.5 B/pixel: what a decoder emits; the
// device converts with rv_nv12_to_bgr_u8) or as raw BGR.
//
// Formats: YUV4MPEG2 (.y4m, 4:2:0 planar, converted to NV12 by the reader
// thread: U/V interleave), raw NV12, raw BGR.  There is no bitstream decoder
// in this image (no rocDecode), and no V4L2 camera: DESIGN.md §(f)4.
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <stdlib.h>
#include <string.h>

#include "common.h"

namespace rv {

namespace {

struct CapSlot {
  uint8_t* p = nullptr;
  double ts = 0.0;
  int64_t index = -1;
  int state = 0;  // 0 free, 1 filled, 2 held by the consumer
  bool pinned = false;
};

struct Capture {
  FILE* f = nullptr;
  int fmt = 0, W = 0, H = 0;
  size_t frame_bytes = 0;  // bytes handed out per frame (NV12 or BGR)
  long data_start = 0;
  bool loop = false, pinned = false;
  std::vector<CapSlot> slots;
  std::vector<uint8_t> uv;  // Y4M: one frame's U and V planes
  int head = 0, tail = 0;
  std::mutex m;
  std::condition_variable cv_fill, cv_take;
  std::thread th;
  bool stop = false, eof = false;
  int err = RV_OK;
  int64_t count = 0;
  // uploaded slots whose H2D copy may still be in flight (consumer side):
  // the slot goes back to the reader when its event has completed
  struct InFlight {
    hipEvent_t ev;
    int slot;
    hipStream_t st;
  };
  std::deque<InFlight> inflight;
};

double wall_now() {
  using namespace std::chrono;
  return duration<double>(system_clock::now().time_since_epoch()).count();
}

// "YUV4MPEG2 W1920 H1080 F30:1 Ip A1:1 C420jpeg\n": width, height and a
// 4:2:0 colour space (C420, C420jpeg, C420paldv, C420mpeg2, or none).
int parse_y4m_header(Capture* c) {
  char line[512];
  if (!fgets(line, sizeof(line), c->f) || strncmp(line, "YUV4MPEG2 ", 10) != 0) {
    set_error("not a YUV4MPEG2 stream");
    return RV_EINVAL;
  }
  if (!strchr(line, '\n')) {
    set_error("YUV4MPEG2 header longer than 511 bytes");
    return RV_EINVAL;
  }
  int W = 0, H = 0;
  char* save = nullptr;
  for (char* tok = strtok_r(line + 10, " \n", &save); tok; tok = strtok_r(nullptr, " \n", &save)) {
    if (tok[0] == 'W') W = atoi(tok + 1);
    if (tok[0] == 'H') H = atoi(tok + 1);
    if (tok[0] == 'C' && strncmp(tok, "C420", 4) != 0) {
      set_error("YUV4MPEG2 colour space %s: only 4:2:0 is supported", tok);
      return RV_EINVAL;
    }
  }
  if (W <= 0 || H <= 0 || W % 2 || H % 2) {
    set_error("YUV4MPEG2 size %dx%d (need positive even sizes)", W, H);
    return RV_EINVAL;
  }
  c->W = W;
  c->H = H;
  return RV_OK;
}

// One frame into `dst`: 1 = ok, 0 = end of file, < 0 = error.
int read_frame(Capture* c, uint8_t* dst) {
  if (c->fmt == RV_CAP_Y4M) {
    char line[256];
    if (!fgets(line, sizeof(line), c->f)) return 0;
    if (strncmp(line, "FRAME", 5) != 0) {
      set_error("YUV4MPEG2: expected FRAME, got '%.16s'", line);
      return RV_EINVAL;
    }
    const size_t ny = (size_t)c->W * c->H, nc = ny / 4;
    if (fread(dst, 1, ny, c->f) != ny || fread(c->uv.data(), 1, 2 * nc, c->f) != 2 * nc)
      return 0;  // truncated last frame: end of stream
    const uint8_t* u = c->uv.data();
    const uint8_t* v = u + nc;
    uint8_t* d = dst + ny;
    for (size_t i = 0; i < nc; ++i) {  // I420 planes -> NV12 interleaved U,V
      d[2 * i] = u[i];
      d[2 * i + 1] = v[i];
    }
    return 1;
  }
  return fread(dst, 1, c->frame_bytes, c->f) == c->frame_bytes ? 1 : 0;
}

void reader_main(Capture* c) {
  for (;;) {
    int i;
    {
      std::unique_lock<std::mutex> lk(c->m);
      c->cv_fill.wait(lk, [&] { return c->stop || c->slots[c->head].state == 0; });
      if (c->stop) return;
      i = c->head;
    }
    int rc = read_frame(c, c->slots[i].p);
    if (rc == 0 && c->loop && c->count > 0) {
      clearerr(c->f);
      if (fseek(c->f, c->data_start, SEEK_SET) == 0) rc = read_frame(c, c->slots[i].p);
    }
    const double ts = wall_now();
    {
      std::lock_guard<std::mutex> lk(c->m);
      if (rc <= 0) {
        c->eof = true;
        c->err = rc < 0 ? rc : RV_OK;
        c->cv_take.notify_all();
        return;
      }
      CapSlot& s = c->slots[i];
      s.ts = ts;
      s.index = c->count++;
      s.state = 1;
      c->head = (c->head + 1) % (int)c->slots.size();
    }
    c->cv_take.notify_one();
  }
}

// Next filled slot in order (blocking): RV_OK, RV_EOF, or an error.
int take(Capture* c, int* slot) {
  std::unique_lock<std::mutex> lk(c->m);
  c->cv_take.wait(lk, [&] { return c->slots[c->tail].state == 1 || c->eof; });
  CapSlot& s = c->slots[c->tail];
  if (s.state != 1) return c->err != RV_OK ? c->err : RV_EOF;
  s.state = 2;
  *slot = c->tail;
  c->tail = (c->tail + 1) % (int)c->slots.size();
  return RV_OK;
}

void give_back(Capture* c, int slot) {
  {
    std::lock_guard<std::mutex> lk(c->m);
    c->slots[slot].state = 0;
  }
  c->cv_fill.notify_one();
}

// The oldest in-flight copy has finished (or failed): its slot goes back to
// the reader.  On a failed query / wait the copy may still be reading the
// slot, so the stream (then the device) is synchronised before the slot is
// released.  Returns false on an error.
bool retire_front(Capture* c, hipError_t e) {
  Capture::InFlight f = c->inflight.front();
  c->inflight.pop_front();
  bool ok = e == hipSuccess;
  if (!ok) {
    set_error("capture: copy event: %s", hipGetErrorString(e));
    if (hipStreamSynchronize(f.st) != hipSuccess) (void)hipDeviceSynchronize();
    (void)hipGetLastError();
  }
  (void)hipEventDestroy(f.ev);
  give_back(c, f.slot);
  return ok;
}

// Return the slots whose copies have completed, without waiting.
bool reap_done(Capture* c) {
  bool ok = true;
  while (!c->inflight.empty()) {
    const hipError_t e = hipEventQuery(c->inflight.front().ev);
    if (e == hipErrorNotReady) break;
    ok = retire_front(c, e) && ok;
  }
  return ok;
}

// Wait for the oldest in-flight copy only and return its slot.
bool reap_oldest(Capture* c) {
  if (c->inflight.empty()) return true;
  return retire_front(c, hipEventSynchronize(c->inflight.front().ev));
}

// take() for the upload path.  The next slot in order (the ring's tail) is
// filled (take it), free (the reader is filling it: take() waits for the
// reader), or still held by an earlier upload whose copy may be in flight --
// the ring has gone all the way round -- and only then the host waits, for
// the oldest copy alone (which is that slot's: copies retire in order).
int take_for_upload(Capture* c, int* slot) {
  if (!reap_done(c)) return RV_EINVAL;
  for (;;) {
    int st;
    bool eof;
    {
      std::lock_guard<std::mutex> lk(c->m);
      st = c->slots[c->tail].state;
      eof = c->eof;
    }
    if (st != 2 || eof || c->inflight.empty()) break;
    if (!reap_oldest(c)) return RV_EINVAL;
  }
  return take(c, slot);
}

}  // namespace

extern "C" int rv_capture_open(const char* path, int fmt, int W, int H, int nbuf, int loop,
                               void** handle) {
  RV_CHECK_ARG(path != nullptr && handle != nullptr, "null pointer");
  RV_CHECK_ARG(fmt == RV_CAP_Y4M || fmt == RV_CAP_NV12 || fmt == RV_CAP_BGR, "format %d", fmt);
  RV_CHECK_ARG(nbuf >= 2 && nbuf <= 64, "nbuf %d out of [2, 64]", nbuf);
  *handle = nullptr;
  Capture* c = new Capture();
  c->fmt = fmt;
  c->loop = loop != 0;
  c->f = fopen(path, "rb");
  if (!c->f) {
    delete c;
    set_error("cannot open %s", path);
    return RV_EINVAL;
  }
  int rc = RV_OK;
  if (fmt == RV_CAP_Y4M) {
    rc = parse_y4m_header(c);
  } else if (W <= 0 || H <= 0 || (fmt == RV_CAP_NV12 && (W % 2 || H % 2))) {
    set_error("raw frames need a positive size (NV12: even) %dx%d", W, H);
    rc = RV_EINVAL;
  } else {
    c->W = W;
    c->H = H;
  }
  if (rc != RV_OK) {
    fclose(c->f);
    delete c;
    return rc;
  }
  c->data_start = ftell(c->f);
  const size_t px = (size_t)c->W * c->H;
  c->frame_bytes = fmt == RV_CAP_BGR ? 3 * px : px + px / 2;
  if (fmt == RV_CAP_Y4M) c->uv.resize(px / 2);
  c->slots.resize(nbuf);
  int dev_count = 0;
  c->pinned = hipGetDeviceCount(&dev_count) == hipSuccess && dev_count > 0;
  for (auto& s : c->slots) {
    void* p = nullptr;
    if (c->pinned && hipHostMalloc(&p, c->frame_bytes, hipHostMallocDefault) != hipSuccess) {
      p = nullptr;
      c->pinned = false;
    }
    s.pinned = p != nullptr;
    if (!p && posix_memalign(&p, 4096, c->frame_bytes) != 0) p = nullptr;
    if (!p) {
      set_error("host slot allocation (%zu bytes) failed", c->frame_bytes);
      for (auto& t : c->slots) {
        if (t.p && t.pinned) (void)hipHostFree(t.p);
        if (t.p && !t.pinned) free(t.p);
      }
      fclose(c->f);
      delete c;
      return RV_EINVAL;
    }
    s.p = (uint8_t*)p;
  }
  c->th = std::thread(reader_main, c);
  *handle = c;
  return RV_OK;
}

extern "C" int rv_capture_info(void* handle, int* info) {
  RV_CHECK_ARG(handle != nullptr && info != nullptr, "null pointer");
  Capture* c = static_cast<Capture*>(handle);
  info[0] = c->W;
  info[1] = c->H;
  info[2] = c->fmt;
  info[3] = (int)c->frame_bytes;
  info[4] = c->slots[0].pinned ? 1 : 0;
  info[5] = (int)c->slots.size();
  return RV_OK;
}

extern "C" int rv_capture_next(void* handle, uint8_t** frame, double* ts, int64_t* index,
                               int* slot) {
  RV_CHECK_ARG(handle != nullptr && frame != nullptr && slot != nullptr, "null pointer");
  Capture* c = static_cast<Capture*>(handle);
  const int rc = take(c, slot);
  if (rc != RV_OK) return rc;
  *frame = c->slots[*slot].p;
  if (ts) *ts = c->slots[*slot].ts;
  if (index) *index = c->slots[*slot].index;
  return RV_OK;
}

extern "C" int rv_capture_release(void* handle, int slot) {
  RV_CHECK_ARG(handle != nullptr, "null pointer");
  Capture* c = static_cast<Capture*>(handle);
  RV_CHECK_ARG(slot >= 0 && slot < (int)c->slots.size() && c->slots[slot].state == 2,
               "slot %d is not held", slot);
  give_back(c, slot);
  return RV_OK;
}

extern "C" int rv_capture_upload_batch(void* const* handles, int S, uint8_t* dev,
                                       size_t dev_stride, double* ts, int64_t* index,
                                       void* stream) {
  RV_CHECK_ARG(handles != nullptr && dev != nullptr && S >= 1, "bad arguments");
  hipStream_t st = as_stream(stream);
  for (int s = 0; s < S; ++s) {
    Capture* c = static_cast<Capture*>(handles[s]);
    RV_CHECK_ARG(c != nullptr && dev_stride >= c->frame_bytes, "stream %d: null or stride", s);
    int slot = -1;
    const int rc = take_for_upload(c, &slot);
    if (rc != RV_OK) return rc;  // frames already queued return their slots at the next reap
    if (ts) ts[s] = c->slots[slot].ts;
    if (index) index[s] = c->slots[slot].index;
    int e = hip_check(hipMemcpyAsync(dev + (size_t)s * dev_stride, c->slots[slot].p,
                                     c->frame_bytes, hipMemcpyHostToDevice, st),
                      "hipMemcpyAsync(capture)");
    hipEvent_t ev = nullptr;
    if (e == RV_OK)
      e = hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate(capture)");
    if (e == RV_OK) e = hip_check(hipEventRecord(ev, st), "hipEventRecord(capture)");
    if (e != RV_OK) {
      if (ev) {
        (void)hipStreamSynchronize(st);
        (void)hipEventDestroy(ev);
      }
      give_back(c, slot);
      return e;
    }
    c->inflight.push_back({ev, slot, st});
  }
  return RV_OK;
}

extern "C" int rv_capture_close(void* handle) {
  if (!handle) return RV_OK;
  Capture* c = static_cast<Capture*>(handle);
  // copies still in flight read the slots: drain every one of them (whatever
  // a wait returns) before the slots are freed
  while (!c->inflight.empty()) (void)reap_oldest(c);
  {
    std::lock_guard<std::mutex> lk(c->m);
    c->stop = true;
  }
  c->cv_fill.notify_all();
  if (c->th.joinable()) c->th.join();
  for (auto& s : c->slots) {
    if (!s.p) continue;
    if (s.pinned)
      (void)hipHostFree(s.p);
    else
      free(s.p);
  }
  if (c->f) fclose(c->f);
  delete c;
  return RV_OK;
}

}  // namespace rv
