#pragma once
#include <hip/hip_runtime.h>
#include <string>
namespace hcu {
bool timing_on();
// Layer tag appended to the kernel name ("kernel@tag") when detail is on.
void timing_set_tag(const char *tag);
int timing_begin(hipStream_t s, const std::string &name, double flops, double bytes);
void timing_end(hipStream_t s, int ev);
// Bracket one launch statement with timing events when timing is enabled.
#define HCU_TIMED(stream, name, flops, bytes, stmt)                        \
  do {                                                                     \
    const int ev__ = ::hcu::timing_on()                                    \
                         ? ::hcu::timing_begin((stream), (name), (flops), (bytes)) \
                         : -1;                                             \
    stmt;                                                                  \
    ::hcu::timing_end((stream), ev__);                                     \
  } while (0)
}  // namespace hcu
