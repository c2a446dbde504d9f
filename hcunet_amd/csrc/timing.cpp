// Opt-in per-launch HIP-event timing (used by bench.py for the roofline).
// When enabled, every kernel launch of the library is bracketed by two
// hipEventRecord()s on the launch stream and tagged with the kernel symbol
// and its algorithmic FLOPs and bytes.  Events come from a pool created at
// enable time, so the timed region performs no allocation.
#include "common.h"
#include "timing.h"
#include "../../include/hcunet.h"
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

namespace hcu {
namespace {
struct Rec {
  std::string name;
  double flops, bytes;
  int ev;
};
std::mutex g_mu;
bool g_on = false;
bool g_detail = false;
thread_local std::string g_tag;
thread_local std::string g_prefix;   // hcu_timing_prefix: the calling chain's name
std::vector<hipEvent_t> g_pool;
std::vector<Rec> g_recs;
size_t g_next = 0;
}  // namespace

bool timing_on() { return g_on; }

// ---- HCU_HOST_PROF=1: host time of kernel launches, other HIP calls and the
// whole forward / backward enqueue (diagnostics; printed to stderr at exit)
namespace {
struct HostProf {
  // [0] launches, [1] other HIP calls (all calls); per steady-state call of
  // the forward / backward (from the 6th on): its launches and HIP calls
  double us[4] = {0, 0, 0, 0};
  long n[4] = {0, 0, 0, 0};
  double in_us[2][3] = {{0, 0, 0}, {0, 0, 0}};   // [fwd|bwd][launch, hip, total]
  long in_n[2][3] = {{0, 0, 0}, {0, 0, 0}};
  long seen[2] = {0, 0};
  ~HostProf() {
    if (n[2] + n[3] == 0) return;
    const char *what[4] = {"kernel launches", "other HIP calls", "hcu_unet_forward", "hcu_unet_backward"};
    for (int k = 0; k < 4; ++k)
      fprintf(stderr, "[hcu host] %-18s %8ld calls %10.1f us total %7.2f us/call\n", what[k], n[k], us[k],
              n[k] ? us[k] / n[k] : 0.0);
    const char *ph[2] = {"forward", "backward"};
    for (int f = 0; f < 2; ++f) {
      const long c = in_n[f][2];
      if (!c) continue;
      fprintf(stderr,
              "[hcu host] steady %s (%ld calls): %.1f us per call; launches %.1f per call, %.1f us; "
              "other HIP calls %.1f per call, %.1f us\n",
              ph[f], c, in_us[f][2] / c, (double)in_n[f][0] / c, in_us[f][0] / c, (double)in_n[f][1] / c,
              in_us[f][1] / c);
    }
  }
};
HostProf g_hp;
const bool g_hp_on = [] {
  const char *e = getenv("HCU_HOST_PROF");
  return e && e[0] == '1';
}();
}  // namespace
bool host_prof_on() { return g_hp_on; }
double host_now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
void host_prof_add(int k, double us) {
  g_hp.us[k] += us;
  g_hp.n[k] += 1;
}
// snapshot at the start of a forward (f = 0) / backward (1); returns a token
void host_prof_call(int f, const double snap_us[2], const long snap_n[2], double total_us) {
  if (++g_hp.seen[f] <= 5) return;
  for (int k = 0; k < 2; ++k) {
    g_hp.in_us[f][k] += g_hp.us[k] - snap_us[k];
    g_hp.in_n[f][k] += g_hp.n[k] - snap_n[k];
  }
  g_hp.in_us[f][2] += total_us;
  g_hp.in_n[f][2] += 1;
}
void host_prof_snap(double snap_us[2], long snap_n[2]) {
  for (int k = 0; k < 2; ++k) {
    snap_us[k] = g_hp.us[k];
    snap_n[k] = g_hp.n[k];
  }
}

void timing_set_tag(const char *tag) {
  if (g_on) g_tag = (g_prefix.empty() ? std::string() : g_prefix + ":") + (tag ? tag : "");
}

int timing_begin(hipStream_t s, const std::string &name, double flops, double bytes) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_on || g_next + 2 > g_pool.size()) return -1;
  const int ev = (int)g_next;
  g_next += 2;
  (void)hipEventRecord(g_pool[ev], s);
  g_recs.push_back(Rec{g_detail && !g_tag.empty() ? name + "@" + g_tag : name, flops, bytes, ev});
  return ev;
}

void timing_end(hipStream_t s, int ev) {
  if (ev < 0) return;
  (void)hipEventRecord(g_pool[ev + 1], s);
}

}  // namespace hcu

using namespace hcu;

extern "C" {

int hcu_timing_enable(int max_launches) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto e : g_pool) (void)hipEventDestroy(e);
  g_pool.clear();
  g_recs.clear();
  g_next = 0;
  g_pool.resize((size_t)max_launches * 2);
  for (auto &e : g_pool) HCU_HIP(hipEventCreate(&e));
  g_on = true;
  return HCU_OK;
}

int hcu_timing_detail(int on) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_detail = on != 0;
  return HCU_OK;
}

int hcu_timing_prefix(const char *prefix) {
  g_prefix = prefix ? prefix : "";
  return HCU_OK;
}

int hcu_timing_disable(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_on = false;
  return HCU_OK;
}

// Synchronises the recorded events and writes one line per kernel symbol:
// "name\tcount\ttotal_ms\tflops\tbytes\n" (totals over launches), then
// clears the records.  Returns the number of bytes needed (excluding NUL).
int64_t hcu_timing_report(char *buf, int64_t len) {
  std::lock_guard<std::mutex> lk(g_mu);
  struct Agg { long n = 0; double ms = 0, fl = 0, by = 0; };
  std::map<std::string, Agg> agg;
  for (const Rec &r : g_recs) {
    (void)hipEventSynchronize(g_pool[r.ev + 1]);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, g_pool[r.ev], g_pool[r.ev + 1]);
    Agg &a = agg[r.name];
    a.n += 1;
    a.ms += ms;
    a.fl += r.flops;
    a.by += r.bytes;
  }
  std::string out;
  char line[512];
  for (const auto &kv : agg) {
    snprintf(line, sizeof line, "%s\t%ld\t%.6f\t%.6e\t%.6e\n", kv.first.c_str(), kv.second.n,
             kv.second.ms, kv.second.fl, kv.second.by);
    out += line;
  }
  if (!buf || len <= 0) return (int64_t)out.size();  // size query: keep the records
  g_recs.clear();
  g_next = 0;
  {
    const size_t n = std::min((size_t)len - 1, out.size());
    std::memcpy(buf, out.data(), n);
    buf[n] = 0;
  }
  return (int64_t)out.size();
}

}  // extern "C"
