// Opt-in per-launch HIP-event timing (used by bench.py for the roofline).
// When enabled, every kernel launch of the library is bracketed by two
// hipEventRecord()s on the launch stream and tagged with the kernel symbol
// and its algorithmic FLOPs and bytes.  Events come from a pool created at
// enable time, so the timed region performs no allocation.
#include "common.h"
#include "timing.h"
#include "../../include/hcunet.h"
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
