// ABI housekeeping: version and thread-local last-error text.
#include <execinfo.h>
#include <signal.h>
#include <stdarg.h>
#include <string.h>
#include <unistd.h>
#include "common.h"

namespace rv {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace rv

extern "C" int rv_abi_version(void) { return 6; }
extern "C" const char* rv_last_error(void) { return rv::g_err; }

// Trace marker: an empty one-wave kernel whose dispatch brackets a region of
// a rocprofv3 kernel trace (bench.py launches tag 1 right before its timed
// region and tag 2 right after it; tools/trace_window.py keeps the kernels
// between them).  No reference counterpart: measurement plumbing only.
__global__ void rv_trace_marker_kernel(int tag) { (void)tag; }

// The marker's grid is `tag` workgroups of 64, so a kernel trace's
// Grid_Size_X (= 64 * tag) names the tag (tools/trace_window.py).
extern "C" int rv_trace_marker(int tag, void* stream) {
  RV_CHECK_ARG(tag >= 1 && tag <= 64, "rv_trace_marker: tag %d outside [1, 64]", tag);
  rv_trace_marker_kernel<<<tag, 64, 0, rv::as_stream(stream)>>>(tag);
  return rv::launch_status("rv_trace_marker");
}

// Native crash report: on SIGSEGV / SIGBUS / SIGABRT / SIGILL / SIGFPE write
// the C stack (backtrace_symbols_fd: module + offset, resolvable offline with
// llvm-symbolizer / nm against the same image) to stderr, then hand the
// signal to the handler that was installed before (Python's faulthandler,
// which adds the Python stack) -- so a host-side fault inside the HIP
// runtime names the frame it died in.  Async-signal-safe calls only.
namespace {
struct sigaction g_prev[32];
bool g_have_prev[32];
char g_altstack[1 << 16];

void crash_handler(int sig, siginfo_t* info, void* uctx) {
  static volatile sig_atomic_t busy = 0;
  if (!busy) {
    busy = 1;
    char head[160];
    const int n = snprintf(head, sizeof(head),
                           "\n[rvhip] fatal signal %d (fault address %p); native stack:\n", sig,
                           info ? info->si_addr : nullptr);
    if (n > 0) (void)!write(2, head, (size_t)n);
    void* frames[64];
    const int nf = backtrace(frames, 64);
    backtrace_symbols_fd(frames, nf, 2);
    (void)!write(2, "[rvhip] end of native stack\n", 28);
  }
  struct sigaction& p = g_prev[sig];
  if (g_have_prev[sig] && (p.sa_flags & SA_SIGINFO) && p.sa_sigaction) {
    p.sa_sigaction(sig, info, uctx);
    return;
  }
  if (g_have_prev[sig] && p.sa_handler != SIG_DFL && p.sa_handler != SIG_IGN &&
      !(p.sa_flags & SA_SIGINFO)) {
    p.sa_handler(sig);
    return;
  }
  signal(sig, SIG_DFL);  // default action: terminate (core) with the same signal
  raise(sig);
}
}  // namespace

extern "C" int rv_install_crash_handler(void) {
  static bool done = false;
  if (done) return RV_OK;
  stack_t ss;
  memset(&ss, 0, sizeof(ss));
  ss.ss_sp = g_altstack;
  ss.ss_size = sizeof(g_altstack);
  (void)sigaltstack(&ss, nullptr);
  void* warm[2];
  (void)backtrace(warm, 2);  // loads libgcc's unwinder now, not inside the handler
  const int sigs[] = {SIGSEGV, SIGBUS, SIGABRT, SIGILL, SIGFPE};
  for (int sig : sigs) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = crash_handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK | SA_NODEFER;
    sigemptyset(&sa.sa_mask);
    g_have_prev[sig] = sigaction(sig, &sa, &g_prev[sig]) == 0;
  }
  done = true;
  return RV_OK;
}
