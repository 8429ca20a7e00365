// Per-process log files and native log lines.
//
// Reference role: the logging java agent (core/agent/src/main/java/org/apache/spark/raydp/
// Agent.java:41-97): every worker process logs into its own file under the session log
// directory, and the file's first line is ":job_id:<id>" so a log monitor can attribute it to
// its job. The supervisor opens an actor's file with rx_log_open before exec'ing the actor,
// so the header is written once per file and every (re)start adds a start line.
#pragma once
#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

namespace rx_log {

inline void stamp(char* buf, size_t n) {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  struct tm tmv;
  localtime_r(&tv.tv_sec, &tmv);
  size_t k = strftime(buf, n, "%Y-%m-%d %H:%M:%S", &tmv);
  snprintf(buf + k, n - k, ".%03d", (int)(tv.tv_usec / 1000));
}

// Open (append) a process log file; an empty file first gets the ":job_id:<id>" header.
inline int open_file(const char* path, const char* job_id, const char* who, int restarts) {
  int fd = open(path, O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
  if (fd < 0) return -1;
  struct stat st;
  char line[512];
  if (fstat(fd, &st) == 0 && st.st_size == 0 && job_id && job_id[0]) {
    int n = snprintf(line, sizeof(line), ":job_id:%s\n", job_id);
    if (write(fd, line, (size_t)n) < 0) { /* best effort */ }
  }
  char ts[64];
  stamp(ts, sizeof(ts));
  int n = snprintf(line, sizeof(line), "[%s] ---- %s start (pid %d, restart %d) ----\n", ts, who, (int)getpid(), restarts);
  if (write(fd, line, (size_t)n) < 0) { /* best effort */ }
  return fd;
}

// "[time] [component pid] message" on stderr (the service's log file).
inline void msg(const char* component, const char* fmt, ...) {
  char ts[64];
  stamp(ts, sizeof(ts));
  char body[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(body, sizeof(body), fmt, ap);
  va_end(ap);
  fprintf(stderr, "[%s] [%s %d] %s\n", ts, component, (int)getpid(), body);
  fflush(stderr);
}

}  // namespace rx_log
