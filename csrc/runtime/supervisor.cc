// Actor supervisor of a runtime node: spawns actor worker processes, watches them, restarts
// the ones that die (bounded by their max_restarts), kills them on request, and tears the whole
// tree down when its parent (the driver) goes away.
//
// Reference roles: Ray's raylet worker pool + GCS actor manager as RayDP uses them — executor
// actors created with max_restarts (RayAppMaster.scala:212-244, the restarted executor asking
// for a new id via RayDPExecutor.scala:121-133), ray.kill(actor, no_restart) in
// RayAppMaster.scala:300-318, and the py4j gateway launcher that dies with its parent
// (AppMasterEntryPoint.scala:36-55 "parent EOF" handshake).
//
// Wire format on the Unix-domain control socket (one request -> one reply, except SUBSCRIBE
// connections, which afterwards receive pushed events):
//   frame  = u32 payload_len | payload
//   payload= u32 op | u32 nstr | nstr x (u32 len | bytes)
// Ops: 1 SPAWN  [id, max_restarts, cwd, log_path, argc, argv..., envc, env...] -> [ok, pid]
//      2 KILL   [id, no_restart, signal]                                      -> [ok] | [err, msg]
//      3 LIST   []                                   -> [id:pid:state:restarts ...]
//      4 SUBSCRIBE []                                -> [ok], then events
//           [died, id, pid, status, will_restart] / [restarted, id, pid, restarts]
//      5 SHUTDOWN []                                 -> [ok] and exit
//      6 PING   []                                   -> [pong]
//      7 WAIT   [id, timeout_ms]  -> [dead, status] | [alive]   (blocks until the process is dead)
// Usage: raydp_supervisor <socket_path>   (exits when stdin reaches EOF)
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/prctl.h>
#include <sys/signalfd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <map>
#include <string>
#include <vector>

#include "logging.h"
#include "trace.h"

namespace {

enum Op : uint32_t { kSpawn = 1, kKill = 2, kList = 3, kSubscribe = 4, kShutdown = 5, kPing = 6, kWait = 7, kEvent = 100, kReply = 101 };

struct Proc {
  std::string id, cwd, log;
  std::vector<std::string> argv, env;
  pid_t pid = -1;
  int max_restarts = 0;  // -1: unlimited
  int restarts = 0;
  bool no_restart = false;
  bool alive = false;
  int status = 0;
};

struct Client {
  int fd;
  std::string in;
  bool subscriber = false;
  // pending WAIT: (proc id, deadline ms)
  std::string wait_id;
  int64_t wait_deadline = 0;
};

std::map<std::string, Proc> g_procs;
std::map<pid_t, std::string> g_by_pid;
std::vector<Client> g_clients;
pid_t g_self;

int64_t now_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000 + ts.tv_nsec / 1000000;
}

void put_u32(std::string& s, uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }

std::string frame(uint32_t op, const std::vector<std::string>& strs) {
  std::string p;
  put_u32(p, op);
  put_u32(p, (uint32_t)strs.size());
  for (const auto& x : strs) {
    put_u32(p, (uint32_t)x.size());
    p += x;
  }
  std::string f;
  put_u32(f, (uint32_t)p.size());
  return f + p;
}

bool write_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t n = write(fd, s.data() + off, s.size() - off);
    if (n < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) {
        pollfd p{fd, POLLOUT, 0};
        poll(&p, 1, 1000);
        continue;
      }
      return false;
    }
    off += (size_t)n;
  }
  return true;
}

bool parse(const std::string& payload, uint32_t* op, std::vector<std::string>* out) {
  if (payload.size() < 8) return false;
  const char* p = payload.data();
  size_t n = payload.size(), off = 8;
  uint32_t cnt;
  memcpy(op, p, 4);
  memcpy(&cnt, p + 4, 4);
  out->clear();
  for (uint32_t i = 0; i < cnt; ++i) {
    if (off + 4 > n) return false;
    uint32_t len;
    memcpy(&len, p + off, 4);
    off += 4;
    if (off + len > n) return false;
    out->emplace_back(p + off, len);
    off += len;
  }
  return true;
}

void broadcast(const std::vector<std::string>& ev) {
  std::string f = frame(kEvent, ev);
  for (auto& c : g_clients)
    if (c.subscriber) write_all(c.fd, f);
}

pid_t spawn(Proc& pr) {
  pid_t pid = fork();
  if (pid < 0) return -1;
  if (pid == 0) {
    setpgid(0, 0);
    prctl(PR_SET_PDEATHSIG, SIGKILL);
    if (getppid() != g_self) _exit(127);
    sigset_t all;
    sigemptyset(&all);
    sigprocmask(SIG_SETMASK, &all, nullptr);
    if (!pr.cwd.empty() && chdir(pr.cwd.c_str()) != 0) _exit(126);
    if (!pr.log.empty()) {
      // per-process log file with the ":job_id:" header (logging agent, Agent.java:41-97)
      std::string job;
      for (const auto& e : pr.env)
        if (e.compare(0, 13, "RAYDP_JOB_ID=") == 0) job = e.substr(13);
      int fd = rx_log::open_file(pr.log.c_str(), job.c_str(), pr.id.c_str(), pr.restarts);
      if (fd >= 0) {
        dup2(fd, 1);
        dup2(fd, 2);
        close(fd);
      }
    }
    int devnull = open("/dev/null", O_RDONLY);
    if (devnull >= 0) {
      dup2(devnull, 0);
      close(devnull);
    }
    std::vector<std::string> env = pr.env;
    env.push_back("RAYDP_ACTOR_RESTART_COUNT=" + std::to_string(pr.restarts));
    std::vector<char*> av, ev;
    for (auto& a : pr.argv) av.push_back(const_cast<char*>(a.c_str()));
    av.push_back(nullptr);
    for (auto& e : env) ev.push_back(const_cast<char*>(e.c_str()));
    ev.push_back(nullptr);
    execvpe(av[0], av.data(), ev.data());
    _exit(127);
  }
  setpgid(pid, pid);
  pr.pid = pid;
  pr.alive = true;
  g_by_pid[pid] = pr.id;
  rx_trace::instant("actor", "spawn " + pr.id, "pid " + std::to_string(pid) + " restart " + std::to_string(pr.restarts));
  return pid;
}

void reap() {
  for (;;) {
    int st = 0;
    pid_t pid = waitpid(-1, &st, WNOHANG);
    if (pid <= 0) return;
    auto it = g_by_pid.find(pid);
    if (it == g_by_pid.end()) continue;
    std::string id = it->second;
    g_by_pid.erase(it);
    auto pit = g_procs.find(id);
    if (pit == g_procs.end()) continue;
    Proc& pr = pit->second;
    if (pr.pid != pid) continue;
    pr.alive = false;
    pr.status = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st);
    // a clean exit (status 0) is a voluntary actor exit: never restarted
    bool restart = !pr.no_restart && pr.status != 0 && (pr.max_restarts < 0 || pr.restarts < pr.max_restarts);
    broadcast({"died", id, std::to_string(pid), std::to_string(pr.status), restart ? "1" : "0"});
    rx_trace::instant("actor", "died " + id, "status " + std::to_string(pr.status) + (restart ? " (restarting)" : ""));
    if (restart) {
      pr.restarts += 1;
      if (spawn(pr) > 0) broadcast({"restarted", id, std::to_string(pr.pid), std::to_string(pr.restarts)});
    }
  }
}

void kill_all() {
  for (auto& kv : g_procs)
    if (kv.second.alive) {
      kv.second.no_restart = true;
      kill(-kv.second.pid, SIGTERM);
    }
  int64_t deadline = now_ms() + 3000;
  for (;;) {
    bool any = false;
    for (auto& kv : g_procs) {
      Proc& pr = kv.second;
      if (!pr.alive) continue;
      int st;
      pid_t r = waitpid(pr.pid, &st, WNOHANG);
      if (r == pr.pid || (r < 0 && errno == ECHILD))
        pr.alive = false;
      else
        any = true;
    }
    if (!any) return;
    if (now_ms() > deadline) {
      for (auto& kv : g_procs)
        if (kv.second.alive) kill(-kv.second.pid, SIGKILL);
      for (auto& kv : g_procs)
        if (kv.second.alive) waitpid(kv.second.pid, nullptr, 0);
      return;
    }
    usleep(20000);
  }
}

std::string handle(Client& c, uint32_t op, const std::vector<std::string>& a, bool* quit) {
  switch (op) {
    case kPing:
      return frame(kReply, {"pong"});
    case kSpawn: {
      if (a.size() < 5) return frame(kReply, {"err", "bad spawn request"});
      Proc pr;
      pr.id = a[0];
      pr.max_restarts = atoi(a[1].c_str());
      pr.cwd = a[2];
      pr.log = a[3];
      size_t argc = (size_t)atoi(a[4].c_str()), i = 5;
      if (argc == 0 || i + argc >= a.size() + 1) return frame(kReply, {"err", "bad argv"});
      for (size_t k = 0; k < argc && i < a.size(); ++k) pr.argv.push_back(a[i++]);
      size_t envc = i < a.size() ? (size_t)atoi(a[i++].c_str()) : 0;
      for (size_t k = 0; k < envc && i < a.size(); ++k) pr.env.push_back(a[i++]);
      auto old = g_procs.find(pr.id);
      if (old != g_procs.end() && old->second.alive) return frame(kReply, {"err", "actor id already running"});
      g_procs[pr.id] = pr;
      pid_t pid = spawn(g_procs[pr.id]);
      if (pid < 0) return frame(kReply, {"err", strerror(errno)});
      return frame(kReply, {"ok", std::to_string(pid)});
    }
    case kKill: {
      if (a.size() < 3) return frame(kReply, {"err", "bad kill request"});
      auto it = g_procs.find(a[0]);
      if (it == g_procs.end()) return frame(kReply, {"err", "no such actor"});
      Proc& pr = it->second;
      if (a[1] == "1") pr.no_restart = true;
      if (pr.alive) kill(-pr.pid, atoi(a[2].c_str()));
      return frame(kReply, {"ok"});
    }
    case kList: {
      std::vector<std::string> out;
      for (auto& kv : g_procs)
        out.push_back(kv.first + ":" + std::to_string(kv.second.pid) + ":" + (kv.second.alive ? "ALIVE" : "DEAD") +
                      ":" + std::to_string(kv.second.restarts));
      return frame(kReply, out);
    }
    case kSubscribe:
      c.subscriber = true;
      return frame(kReply, {"ok"});
    case kShutdown:
      *quit = true;
      return frame(kReply, {"ok"});
    case kWait: {
      if (a.size() < 2) return frame(kReply, {"err", "bad wait"});
      auto it = g_procs.find(a[0]);
      if (it == g_procs.end() || !it->second.alive)
        return frame(kReply, {"dead", it == g_procs.end() ? "-1" : std::to_string(it->second.status)});
      c.wait_id = a[0];
      c.wait_deadline = now_ms() + atoll(a[1].c_str());
      return std::string();  // answered from the main loop
    }
    default:
      return frame(kReply, {"err", "unknown op"});
  }
}

void service_waits() {
  int64_t t = now_ms();
  for (auto& c : g_clients) {
    if (c.wait_id.empty()) continue;
    auto it = g_procs.find(c.wait_id);
    bool dead = it == g_procs.end() || !it->second.alive;
    if (dead || t >= c.wait_deadline) {
      write_all(c.fd, dead ? frame(kReply, {"dead", it == g_procs.end() ? "-1" : std::to_string(it->second.status)})
                           : frame(kReply, {"alive"}));
      c.wait_id.clear();
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <socket_path>\n", argv[0]);
    return 2;
  }
  g_self = getpid();
  signal(SIGPIPE, SIG_IGN);
  sigset_t mask;
  sigemptyset(&mask);
  sigaddset(&mask, SIGCHLD);
  sigaddset(&mask, SIGTERM);
  sigaddset(&mask, SIGINT);
  sigprocmask(SIG_BLOCK, &mask, nullptr);
  int sfd = signalfd(-1, &mask, SFD_CLOEXEC | SFD_NONBLOCK);

  const char* path = argv[1];
  unlink(path);
  int lfd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_un addr{};
  addr.sun_family = AF_UNIX;
  if (strlen(path) >= sizeof(addr.sun_path)) {
    fprintf(stderr, "socket path too long\n");
    return 2;
  }
  strcpy(addr.sun_path, path);
  if (bind(lfd, (sockaddr*)&addr, sizeof(addr)) != 0 || listen(lfd, 128) != 0) {
    perror("bind/listen");
    return 1;
  }
  // handshake: tell the parent we are ready
  write_all(1, "READY\n");

  bool quit = false;
  while (!quit) {
    std::vector<pollfd> fds;
    fds.push_back({0, POLLIN, 0});
    fds.push_back({lfd, POLLIN, 0});
    fds.push_back({sfd, POLLIN, 0});
    for (auto& c : g_clients) fds.push_back({c.fd, POLLIN, 0});
    int timeout = -1;
    for (auto& c : g_clients)
      if (!c.wait_id.empty()) timeout = 50;
    int r = poll(fds.data(), fds.size(), timeout);
    if (r < 0 && errno != EINTR) break;
    if (fds[0].revents & (POLLIN | POLLHUP | POLLERR)) {
      char buf[256];
      ssize_t n = read(0, buf, sizeof(buf));
      if (n <= 0) break;  // parent gone: tear everything down
    }
    if (fds[2].revents & POLLIN) {
      signalfd_siginfo si;
      while (read(sfd, &si, sizeof(si)) == (ssize_t)sizeof(si)) {
        if (si.ssi_signo == SIGTERM || si.ssi_signo == SIGINT) quit = true;
      }
      reap();
    }
    if (fds[1].revents & POLLIN) {
      int cfd = accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
      if (cfd >= 0) g_clients.push_back({cfd});
    }
    std::vector<int> dead;
    for (size_t k = 3; k < fds.size(); ++k) {
      if (!(fds[k].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      Client* c = nullptr;
      for (auto& cc : g_clients)
        if (cc.fd == fds[k].fd) c = &cc;
      if (!c) continue;
      char buf[65536];
      ssize_t n = read(c->fd, buf, sizeof(buf));
      if (n <= 0) {
        dead.push_back(c->fd);
        continue;
      }
      c->in.append(buf, (size_t)n);
      while (c->in.size() >= 4) {
        uint32_t len;
        memcpy(&len, c->in.data(), 4);
        if (c->in.size() < 4 + (size_t)len) break;
        std::string payload = c->in.substr(4, len);
        c->in.erase(0, 4 + (size_t)len);
        uint32_t op;
        std::vector<std::string> args;
        std::string reply = parse(payload, &op, &args) ? handle(*c, op, args, &quit) : frame(kReply, {"err", "bad frame"});
        if (!reply.empty()) write_all(c->fd, reply);
      }
    }
    service_waits();
    for (int fd : dead) {
      close(fd);
      for (size_t i = 0; i < g_clients.size(); ++i)
        if (g_clients[i].fd == fd) {
          g_clients.erase(g_clients.begin() + (long)i);
          break;
        }
    }
  }
  kill_all();
  for (auto& c : g_clients) close(c.fd);
  close(lfd);
  unlink(path);
  return 0;
}
