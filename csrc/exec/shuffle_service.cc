// Per-node external shuffle-block service.
//
// Reference role: RayExternalShuffleService.scala:26-56 + ExternalShuffleServiceUtils.java:26-42
// (Spark's ExternalShuffleService wrapped in an actor pinned to a node, started by the app
// master for every node that hosts an executor when spark.shuffle.service.enabled is set,
// RayAppMaster.scala:155-163). Its point: map outputs outlive the executor that wrote them,
// so executors can be killed (dynamic allocation) or lost without losing finished map work.
//
// Design: a map task hash-partitions its partition into R buckets and writes them, one Arrow
// IPC stream after another, into ONE file under this service's data directory; it registers
// (shuffle, map, path, R+1 offsets). From then on the service owns the file: it keeps it open,
// and a reducer's FETCH gets back (offset, length) plus the file descriptor itself over
// SCM_RIGHTS, so the reducer mmaps the bucket — no byte goes through this process or a socket.
//
// Wire format: csrc/common/frame.h. Requests -> reply op 101:
//   1 REGISTER_OUTPUT [shuffle_id, map_id, path, offsets(csv, R+1)] -> [ok]
//   2 FETCH           [shuffle_id, map_id, reduce_id]  -> [ok, offset, length] + fd | [missing]
//   3 REMOVE_SHUFFLE  [shuffle_id]                      -> [ok, n_files_removed]
//   4 LIST            []                                -> [ok, "sid:mid:buckets:bytes"...]
//   5 DATA_DIR        []                                -> [ok, dir]
//   6 PING -> [pong]    7 SHUTDOWN -> [ok] and exit
// Usage: raydp_shuffle_service <socket_path> <data_dir>     (SIGTERM: remove files, exit)
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/stat.h>

#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "frame.h"
#include "trace.h"

namespace {

using rx_frame::Msg;

enum Op : uint32_t { kRegister = 1, kFetch = 2, kRemove = 3, kList = 4, kDataDir = 5, kPing = 6, kShutdown = 7, kReply = 101 };

struct MapOutput {
  std::string path;
  int fd = -1;
  std::vector<long long> offsets;  // R + 1
};

volatile sig_atomic_t g_stop = 0;
void on_term(int) { g_stop = 1; }

int mkdirs(const std::string& p) {
  std::string cur;
  std::stringstream ss(p);
  std::string part;
  if (!p.empty() && p[0] == '/') cur = "/";
  while (std::getline(ss, part, '/')) {
    if (part.empty()) continue;
    cur += part + "/";
    if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return -1;
  }
  return 0;
}

struct Service {
  std::string dir;
  std::map<std::pair<std::string, long>, MapOutput> outputs;
  bool stop = false;

  Msg reply(std::vector<std::string> s) {
    Msg m;
    m.op = kReply;
    m.s = std::move(s);
    return m;
  }

  int remove_shuffle(const std::string& sid) {
    int n = 0;
    for (auto it = outputs.begin(); it != outputs.end();) {
      if (it->first.first == sid) {
        close(it->second.fd);
        unlink(it->second.path.c_str());
        it = outputs.erase(it);
        ++n;
      } else {
        ++it;
      }
    }
    return n;
  }

  void remove_all() {
    for (auto& kv : outputs) {
      close(kv.second.fd);
      unlink(kv.second.path.c_str());
    }
    outputs.clear();
  }

  // returns the fd to pass along (or -1)
  Msg handle(const Msg& q, int* pass_fd) {
    *pass_fd = -1;
    const auto& a = q.s;
    switch (q.op) {
      case kPing: return reply({"pong"});
      case kDataDir: return reply({"ok", dir});
      case kRegister: {
        if (a.size() < 4) return reply({"err", "bad REGISTER_OUTPUT"});
        MapOutput o;
        o.path = a[2];
        std::stringstream ss(a[3]);
        std::string v;
        while (std::getline(ss, v, ',')) o.offsets.push_back(atoll(v.c_str()));
        if (o.offsets.size() < 2) return reply({"err", "need R+1 offsets"});
        o.fd = open(o.path.c_str(), O_RDONLY | O_CLOEXEC);
        if (o.fd < 0) return reply({"err", std::string("open: ") + strerror(errno)});
        struct stat st;
        if (fstat(o.fd, &st) != 0 || st.st_size < o.offsets.back()) {
          close(o.fd);
          return reply({"err", "file shorter than its index"});
        }
        auto key = std::make_pair(a[0], atol(a[1].c_str()));
        auto old = outputs.find(key);
        if (old != outputs.end()) {  // a re-run map task replaces its output
          close(old->second.fd);
          if (old->second.path != o.path) unlink(old->second.path.c_str());
          outputs.erase(old);
        }
        outputs[key] = o;
        rx_trace::instant("shuffle", "map output " + a[0] + "/" + a[1], std::to_string(o.offsets.back()) + " B");
        return reply({"ok"});
      }
      case kFetch: {
        if (a.size() < 3) return reply({"err", "bad FETCH"});
        auto it = outputs.find(std::make_pair(a[0], atol(a[1].c_str())));
        const long r = atol(a[2].c_str());
        if (it == outputs.end() || r < 0 || r + 1 >= (long)it->second.offsets.size()) return reply({"missing"});
        const long long off = it->second.offsets[r], len = it->second.offsets[r + 1] - off;
        *pass_fd = it->second.fd;
        return reply({"ok", std::to_string(off), std::to_string(len)});
      }
      case kRemove: {
        if (a.empty()) return reply({"err", "bad REMOVE_SHUFFLE"});
        return reply({"ok", std::to_string(remove_shuffle(a[0]))});
      }
      case kList: {
        std::vector<std::string> out = {"ok"};
        for (auto& kv : outputs)
          out.push_back(kv.first.first + ":" + std::to_string(kv.first.second) + ":" +
                        std::to_string(kv.second.offsets.size() - 1) + ":" + std::to_string(kv.second.offsets.back()));
        return reply(out);
      }
      case kShutdown:
        stop = true;
        return reply({"ok"});
      default:
        return reply({"err", "unknown op"});
    }
  }
};

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <socket_path> <data_dir>\n", argv[0]);
    return 2;
  }
  signal(SIGPIPE, SIG_IGN);
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_term;
  sigaction(SIGTERM, &sa, nullptr);
  Service s;
  s.dir = argv[2];
  if (mkdirs(s.dir) != 0) {
    perror("shuffle_service: data dir");
    return 1;
  }
  int lfd = rx_frame::listen_unix(argv[1]);
  if (lfd < 0) {
    perror("shuffle_service: listen");
    return 1;
  }
  std::vector<int> conns;
  while (!s.stop && !g_stop) {
    std::vector<struct pollfd> fds;
    fds.push_back({lfd, POLLIN, 0});
    for (int c : conns) fds.push_back({c, POLLIN, 0});
    int r = poll(fds.data(), fds.size(), 500);
    if (r < 0) {
      if (errno == EINTR) continue;
      break;
    }
    if (fds[0].revents & POLLIN) {
      int c = accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
      if (c >= 0) conns.push_back(c);
    }
    std::vector<int> dead;
    for (size_t i = 1; i < fds.size(); ++i) {
      if (!(fds[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      Msg q;
      if (!rx_frame::read_msg(fds[i].fd, q)) {
        dead.push_back(fds[i].fd);
        continue;
      }
      int pass = -1;
      Msg rep = s.handle(q, &pass);
      bool ok = pass >= 0 ? rx_frame::write_msg_fd(fds[i].fd, rep, pass) : rx_frame::write_msg(fds[i].fd, rep);
      if (!ok) dead.push_back(fds[i].fd);
    }
    for (int d : dead) {
      close(d);
      for (size_t i = 0; i < conns.size(); ++i)
        if (conns[i] == d) {
          conns.erase(conns.begin() + i);
          break;
        }
    }
  }
  s.remove_all();
  for (int c : conns) close(c);
  close(lfd);
  unlink(argv[1]);
  return 0;
}
