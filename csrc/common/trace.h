// Chrome-trace events from native services (actor spawn / death / restart, executor
// registration, shuffle map-output registration and fetch).
//
// Enabled when RAYDP_TRACE (config key spark.ray.mi355x.trace) names a trace path: each
// process appends one JSON object per line to "<path>.<pid>.jsonl"; raydp_amd.utils.tracing
// merges those files (Python spans included) into one chrome://tracing / Perfetto JSON.
// Timestamps are CLOCK_REALTIME microseconds, the clock the Python side uses too.
#pragma once
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <string>

namespace rx_trace {

inline FILE* sink() {
  static FILE* f = nullptr;
  static bool init = false;
  if (!init) {
    init = true;
    const char* p = getenv("RAYDP_TRACE");
    if (p && p[0]) {
      std::string path = std::string(p) + "." + std::to_string((int)getpid()) + ".jsonl";
      f = fopen(path.c_str(), "a");
    }
  }
  return f;
}

inline long long now_us() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return (long long)ts.tv_sec * 1000000 + ts.tv_nsec / 1000;
}

inline std::string esc(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    if ((unsigned char)c < 0x20) continue;
    o += c;
  }
  return o;
}

// Instant event ("ph":"i") with one string argument.
inline void instant(const char* cat, const std::string& name, const std::string& arg = "") {
  FILE* f = sink();
  if (!f) return;
  fprintf(f, "{\"name\":\"%s\",\"cat\":\"%s\",\"ph\":\"i\",\"s\":\"p\",\"ts\":%lld,\"pid\":%d,\"tid\":0,\"args\":{\"detail\":\"%s\"}}\n",
          esc(name).c_str(), cat, now_us(), (int)getpid(), esc(arg).c_str());
  fflush(f);
}

// Complete event ("ph":"X") of duration dur_us that started at ts_us.
inline void complete(const char* cat, const std::string& name, long long ts_us, long long dur_us) {
  FILE* f = sink();
  if (!f) return;
  fprintf(f, "{\"name\":\"%s\",\"cat\":\"%s\",\"ph\":\"X\",\"ts\":%lld,\"dur\":%lld,\"pid\":%d,\"tid\":0}\n",
          esc(name).c_str(), cat, ts_us, dur_us, (int)getpid());
  fflush(f);
}

}  // namespace rx_trace
