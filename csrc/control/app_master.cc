// Application master of a Spark-on-runtime application: the native control plane.
//
// Reference roles, re-designed as one single-threaded service process:
//   J1 RayAppMaster.scala        app registration, executor scheduling (requestNewExecutor caps,
//                                 :258-303), RegisterExecutor / ExecutorStarted / RequestExecutors /
//                                 KillExecutors / RequestAddPendingRestartedExecutor (:150-210),
//                                 onDisconnected -> kill bookkeeping without stopping the actor
//                                 (:212-214), one external shuffle service per node (:155-163),
//                                 restarted-executor map (:84, :192-209), master URL (:89-92)
//   J7 ApplicationInfo/-Description/-State   the app model and executor state machine
//   J9 Messages.scala             the op set below
//   J11 RayDPDriverAgent          RecacheRDD is relayed to the driver's event subscription
//   J5 AppMasterEntryPoint        handshake file written via tmp + rename; exits on stdin EOF
//   J10 launch half of RayExternalShuffleService / ExternalShuffleServiceUtils (fork/exec of
//                                 the native raydp_shuffle_service binary)
//
// The master decides WHAT to launch; the driver's runtime creates the actor processes
// (RayExecutorUtils.createExecutorActor's role) from the launch orders the master returns,
// each order carrying executor id, CPU, memory, custom resources and placement bundle.
// Executors keep their registration connection open for life: its EOF is the disconnect.
//
// Wire format: csrc/common/frame.h. Requests (op [args]) -> reply op 101 [status, ...]:
//   1  REGISTER_APP   [name, num_executors, cores, memory_mb, actor_cpu, user, res(k=v,..),
//                      bundles(csv), dyn_alloc(0|1), max_executors, shuffle_service(0|1),
//                      local_dir, node_ip]                     -> [ok, app_id, master_url, order...]
//   2  UNREGISTER_APP [app_id]                                  -> [ok]
//   3  REGISTER_EXECUTOR [executor_id, node_id, pid, restarted(0|1)]
//                                          -> [ok, effective_id, shuffle_socket|""] | [err, why]
//   4  EXECUTOR_STARTED [executor_id]                           -> [ok]
//   5  REQUEST_EXECUTORS [app_id, total]                        -> [ok, order...]
//   6  KILL_EXECUTORS [app_id, id...]                           -> [ok|partial, killed_id...]
//   7  GET_RESTARTED  []                                        -> [ok, new=old...]
//   8  APP_INFO       []                                        -> [ok, key=value...]
//   9  RECACHE_RDD    [rdd_id]                                  -> [ok, n_subscribers]
//   10 SUBSCRIBE      []  -> [ok], then pushed events op 100: [recache, rdd_id]
//   11 PING -> [pong]    12 SHUTDOWN -> [ok] and exit    13 MASTER_URL -> [ok, url]
//   14 EXECUTOR_LOST  [executor_id, shutdown_actor(0|1)]        -> [ok|unknown]
// Usage: raydp_appmaster <socket_path> <conn_info_path> [shuffle_service_binary]
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <sys/wait.h>
#include <time.h>

#include <deque>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "frame.h"
#include "logging.h"
#include "trace.h"

namespace {

using rx_frame::Msg;

enum Op : uint32_t {
  kRegisterApp = 1, kUnregisterApp = 2, kRegisterExecutor = 3, kExecutorStarted = 4,
  kRequestExecutors = 5, kKillExecutors = 6, kGetRestarted = 7, kAppInfo = 8, kRecacheRdd = 9,
  kSubscribe = 10, kPing = 11, kShutdown = 12, kMasterUrl = 13, kExecutorLost = 14,
  kEvent = 100, kReply = 101
};

enum class AppState { WAITING, RUNNING, FINISHED, FAILED, KILLED, UNKNOWN };
const char* state_name(AppState s) {
  switch (s) {
    case AppState::WAITING: return "WAITING";
    case AppState::RUNNING: return "RUNNING";
    case AppState::FINISHED: return "FINISHED";
    case AppState::FAILED: return "FAILED";
    case AppState::KILLED: return "KILLED";
    default: return "UNKNOWN";
  }
}

long long now_ms() {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  return (long long)tv.tv_sec * 1000 + tv.tv_usec / 1000;
}

struct AppDesc {  // ApplicationDescription
  std::string name, user, local_dir, node_ip;
  int num_executors = 1, cores = 1, memory_mb = 1024, max_executors = 0;
  double actor_cpu = 1.0;
  bool dyn_alloc = false, shuffle_service = false;
  std::vector<std::pair<std::string, double>> resources;
  std::vector<int> bundles;
};

struct ExecutorDesc {
  std::string id, node, pid;
  int cores = 1, memory_mb = 0, bundle = -1;
  bool registered = false, started = false;
  int conn = -1;  // registration connection (its EOF = disconnect)
};

struct AppInfo {  // ApplicationInfo
  std::string id;
  AppDesc desc;
  AppState state = AppState::WAITING;
  long long start_ms = 0, end_ms = -1;
  std::map<std::string, ExecutorDesc> executors;
  std::vector<std::string> removed;
  int registered = 0;  // registered minus removed
  int next_id = 0;
  int bundle_rr = 0;

  int remaining_unregistered() const { return desc.num_executors - registered; }
  std::string next_executor_id() { return std::to_string(next_id++); }
  bool register_executor(const std::string& id) {
    auto it = executors.find(id);
    if (it == executors.end()) {
      rx_log::msg("appmaster", "register of unknown executor %s", id.c_str());
      return false;
    }
    if (it->second.registered) {
      rx_log::msg("appmaster", "executor %s registered twice", id.c_str());
      return false;
    }
    it->second.registered = true;
    ++registered;
    return true;
  }
  bool kill(const std::string& id) {
    auto it = executors.find(id);
    if (it == executors.end()) return false;
    if (it->second.registered) --registered;
    removed.push_back(id);
    executors.erase(it);
    return true;
  }
  void mark_finished(AppState s) {
    state = s;
    end_ms = now_ms();
  }
  long long duration() const { return (end_ms != -1 ? end_ms : now_ms()) - start_ms; }
};

struct Master {
  std::string sock_path, shuffle_bin;
  int listen_fd = -1;
  bool have_app = false;
  AppInfo app;
  std::map<std::string, std::string> restarted;  // new id -> old id
  std::map<std::string, std::pair<pid_t, std::string>> shuffle_services;  // node -> (pid, socket)
  std::set<int> subscribers;
  bool stop = false;

  std::string master_url() const {
    // RayAppMaster.getMasterUrl: spark://host:port -> ray://; here the endpoint is a socket
    return "ray://" + app.desc.name + "@" + app.desc.node_ip + ":" + std::to_string(getpid());
  }

  std::string order_for(const ExecutorDesc& e) const {
    std::ostringstream o;
    o << "id=" << e.id << ";cpu=" << app.desc.actor_cpu << ";memory_mb=" << e.memory_mb
      << ";cores=" << e.cores << ";bundle=" << e.bundle << ";res=";
    bool first = true;
    for (auto& kv : app.desc.resources) {
      o << (first ? "" : ",") << kv.first << ":" << kv.second;
      first = false;
    }
    return o.str();
  }

  // RayAppMaster.requestNewExecutor: caps count current AND restarted executors.
  bool request_new_executor(std::vector<std::string>& orders) {
    const int have = (int)app.executors.size() + (int)restarted.size();
    if (app.desc.dyn_alloc) {
      if (have >= app.desc.max_executors) return false;
    } else if (app.desc.num_executors != 0 && have >= app.desc.num_executors) {
      return false;
    }
    ExecutorDesc e;
    e.id = app.next_executor_id();
    e.cores = app.desc.cores;
    e.memory_mb = app.desc.memory_mb;
    if (!app.desc.bundles.empty()) e.bundle = app.desc.bundles[app.bundle_rr++ % app.desc.bundles.size()];
    app.executors[e.id] = e;  // addPendingRegisterExecutor
    orders.push_back(order_for(e));
    return true;
  }

  std::string ensure_shuffle_service(const std::string& node) {
    if (!app.desc.shuffle_service || shuffle_bin.empty()) return "";
    auto it = shuffle_services.find(node);
    if (it != shuffle_services.end()) return it->second.second;
    std::string sock = sock_path + ".shuffle." + node;
    std::string dir = app.desc.local_dir.empty() ? sock_path + ".shuffle-data." + node : app.desc.local_dir + "/" + node;
    pid_t pid = fork();
    if (pid == 0) {
      int devnull = open("/dev/null", O_RDONLY);
      if (devnull >= 0) dup2(devnull, 0);  // the service has its own lifetime (killed on stop)
      execl(shuffle_bin.c_str(), shuffle_bin.c_str(), sock.c_str(), dir.c_str(), (char*)nullptr);
      _exit(127);
    }
    if (pid < 0) return "";
    // wait until the socket exists (bounded)
    for (int i = 0; i < 500; ++i) {
      struct stat st;
      if (stat(sock.c_str(), &st) == 0) break;
      usleep(2000);
    }
    rx_log::msg("appmaster", "started shuffle service on node %s (pid %d)", node.c_str(), (int)pid);
    rx_trace::instant("appmaster", "shuffle service " + node, sock);
    shuffle_services[node] = {pid, sock};
    return sock;
  }

  void stop_shuffle_services() {
    for (auto& kv : shuffle_services) {
      kill(kv.second.first, SIGTERM);
      waitpid(kv.second.first, nullptr, 0);
    }
    shuffle_services.clear();
  }

  void on_disconnected(int conn) {
    for (auto& kv : app.executors)
      if (kv.second.conn == conn) {
        rx_log::msg("appmaster", "executor %s disconnected", kv.first.c_str());
        rx_trace::instant("appmaster", "executor disconnected " + kv.first);
        app.kill(kv.first);  // shutdownActor = false: the runtime may restart it
        return;
      }
  }

  Msg reply(std::vector<std::string> s) {
    Msg m;
    m.op = kReply;
    m.s = std::move(s);
    return m;
  }

  Msg handle(int conn, const Msg& q) {
    const auto& a = q.s;
    switch (q.op) {
      case kPing: return reply({"pong"});
      case kMasterUrl: return reply({"ok", master_url()});
      case kRegisterApp: {
        if (a.size() < 13) return reply({"err", "bad REGISTER_APP"});
        if (have_app && app.state == AppState::RUNNING) return reply({"err", "application already registered"});
        AppInfo fresh;
        fresh.start_ms = now_ms();
        char buf[64];
        time_t t = (time_t)(fresh.start_ms / 1000);
        struct tm tmv;
        localtime_r(&t, &tmv);
        strftime(buf, sizeof(buf), "%Y%m%d%H%M%S", &tmv);
        char id[96];
        snprintf(id, sizeof(id), "app-%s%03lld", buf, fresh.start_ms % 1000);
        fresh.id = id;
        AppDesc& d = fresh.desc;
        d.name = a[0];
        d.num_executors = atoi(a[1].c_str());
        d.cores = atoi(a[2].c_str());
        d.memory_mb = atoi(a[3].c_str());
        d.actor_cpu = atof(a[4].c_str());
        d.user = a[5];
        std::stringstream rs(a[6]);
        std::string kv;
        while (std::getline(rs, kv, ',')) {
          size_t eq = kv.find('=');
          if (eq != std::string::npos) d.resources.push_back({kv.substr(0, eq), atof(kv.c_str() + eq + 1)});
        }
        std::stringstream bs(a[7]);
        while (std::getline(bs, kv, ','))
          if (!kv.empty()) d.bundles.push_back(atoi(kv.c_str()));
        d.dyn_alloc = a[8] == "1";
        d.max_executors = atoi(a[9].c_str());
        d.shuffle_service = a[10] == "1";
        d.local_dir = a[11];
        d.node_ip = a[12];
        app = fresh;
        have_app = true;
        restarted.clear();
        app.state = AppState::RUNNING;
        rx_log::msg("appmaster", "registered application %s (%s), %d executors", app.id.c_str(), d.name.c_str(),
                    d.num_executors);
        rx_trace::instant("appmaster", "register application " + app.id, d.name);
        std::vector<std::string> out = {"ok", app.id, master_url()};
        std::vector<std::string> orders;
        for (int i = 0; i < d.num_executors; ++i) request_new_executor(orders);  // schedule()
        out.insert(out.end(), orders.begin(), orders.end());
        return reply(out);
      }
      case kUnregisterApp:
        if (have_app) app.mark_finished(AppState::FINISHED);
        return reply({"ok"});
      case kRegisterExecutor: {
        if (a.size() < 4 || !have_app) return reply({"err", "no application"});
        std::string eid = a[0];
        if (a[3] == "1") {  // RequestAddPendingRestartedExecutor
          if (app.remaining_unregistered() <= 0) return reply({"err", "no slot for a restarted executor"});
          std::string nid = app.next_executor_id();
          ExecutorDesc e;
          e.id = nid;
          e.cores = app.desc.cores;
          e.memory_mb = app.desc.memory_mb;
          app.executors[nid] = e;
          restarted[nid] = eid;
          eid = nid;
        }
        if (!app.register_executor(eid)) return reply({"err", "register rejected"});
        rx_trace::instant("appmaster", "register executor " + eid, a[3] == "1" ? "restarted from " + a[0] : "");
        ExecutorDesc& e = app.executors[eid];
        e.node = a[1];
        e.pid = a[2];
        e.conn = conn;
        const std::string shuffle = ensure_shuffle_service(e.node);
        return reply({"ok", eid, shuffle});
      }
      case kExecutorStarted: {
        if (a.empty()) return reply({"err", "bad EXECUTOR_STARTED"});
        auto it = app.executors.find(a[0]);
        if (it == app.executors.end()) return reply({"err", "unknown executor"});
        it->second.started = true;
        return reply({"ok"});
      }
      case kRequestExecutors: {
        if (a.size() < 2 || !have_app || a[0] != app.id) return reply({"err", "unknown application"});
        const int total = atoi(a[1].c_str());
        std::vector<std::string> out = {"ok"};
        if (total > app.registered) {
          std::vector<std::string> orders;
          // pending (launched, not yet registered) executors already count toward the total
          int pending = 0;
          for (auto& kv : app.executors)
            if (!kv.second.registered) ++pending;
          for (int i = 0; i < total - app.registered - pending; ++i)
            if (!request_new_executor(orders)) break;
          out.insert(out.end(), orders.begin(), orders.end());
        }
        return reply(out);
      }
      case kKillExecutors: {
        if (a.empty() || !have_app || a[0] != app.id) return reply({"err", "unknown application"});
        bool all = true;
        std::vector<std::string> killed;
        for (size_t i = 1; i < a.size(); ++i) {
          if (app.kill(a[i]))
            killed.push_back(a[i]);
          else
            all = false;
        }
        std::vector<std::string> out = {all ? "ok" : "partial"};
        out.insert(out.end(), killed.begin(), killed.end());
        return reply(out);
      }
      case kExecutorLost: {
        if (a.empty()) return reply({"err", "bad EXECUTOR_LOST"});
        return reply({app.kill(a[0]) ? "ok" : "unknown"});
      }
      case kGetRestarted: {
        std::vector<std::string> out = {"ok"};
        for (auto& kv : restarted) out.push_back(kv.first + "=" + kv.second);
        return reply(out);
      }
      case kAppInfo: {
        std::vector<std::string> out = {"ok"};
        if (!have_app) return reply({"ok", "state=UNKNOWN"});
        out.push_back("app_id=" + app.id);
        out.push_back("name=" + app.desc.name);
        out.push_back(std::string("state=") + state_name(app.state));
        out.push_back("duration_ms=" + std::to_string(app.duration()));
        out.push_back("registered=" + std::to_string(app.registered));
        out.push_back("remaining_unregistered=" + std::to_string(app.remaining_unregistered()));
        for (auto& kv : app.executors) {
          const ExecutorDesc& e = kv.second;
          out.push_back("executor=" + e.id + ":" + (e.registered ? "registered" : "pending") + ":" +
                        (e.started ? "started" : "-") + ":" + e.node + ":" + std::to_string(e.bundle));
        }
        for (auto& r : app.removed) out.push_back("removed=" + r);
        for (auto& kv : shuffle_services) out.push_back("shuffle_service=" + kv.first + ":" + kv.second.second);
        return reply(out);
      }
      case kRecacheRdd: {
        if (a.empty()) return reply({"err", "bad RECACHE_RDD"});
        Msg ev;
        ev.op = kEvent;
        ev.s = {"recache", a[0]};
        int n = 0;
        for (auto it = subscribers.begin(); it != subscribers.end();) {
          if (rx_frame::write_msg(*it, ev)) {
            ++n;
            ++it;
          } else {
            it = subscribers.erase(it);
          }
        }
        return reply({"ok", std::to_string(n)});
      }
      case kSubscribe:
        subscribers.insert(conn);
        return reply({"ok"});
      case kShutdown:
        stop = true;
        return reply({"ok"});
      default:
        return reply({"err", "unknown op"});
    }
  }
};

int write_handshake(const std::string& path, const std::string& sock) {
  const std::string tmp = path + ".tmp";
  FILE* f = fopen(tmp.c_str(), "w");
  if (!f) return -1;
  fprintf(f, "%s\n%d\n", sock.c_str(), (int)getpid());
  fclose(f);
  return rename(tmp.c_str(), path.c_str());
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <socket_path> <conn_info_path> [shuffle_service_binary]\n", argv[0]);
    return 2;
  }
  signal(SIGPIPE, SIG_IGN);
  signal(SIGINT, SIG_IGN);  // like the reference gateway: only the parent's EOF stops us
  Master m;
  m.sock_path = argv[1];
  if (argc > 3) m.shuffle_bin = argv[3];
  m.listen_fd = rx_frame::listen_unix(m.sock_path);
  if (m.listen_fd < 0) {
    perror("appmaster: listen");
    return 1;
  }
  if (write_handshake(argv[2], m.sock_path) != 0) {
    perror("appmaster: handshake");
    return 1;
  }
  std::vector<int> conns;
  bool stdin_open = true;
  while (!m.stop) {
    std::vector<struct pollfd> fds;
    fds.push_back({m.listen_fd, POLLIN, 0});
    if (stdin_open) fds.push_back({0, POLLIN, 0});
    const size_t base = fds.size();
    for (int c : conns) fds.push_back({c, POLLIN, 0});
    int r = poll(fds.data(), fds.size(), 1000);
    if (r < 0) {
      if (errno == EINTR) continue;
      break;
    }
    if (fds[0].revents & POLLIN) {
      int c = accept4(m.listen_fd, nullptr, nullptr, SOCK_CLOEXEC);
      if (c >= 0) conns.push_back(c);
    }
    if (stdin_open && (fds[1].revents & (POLLIN | POLLHUP | POLLERR))) {
      char buf[256];
      ssize_t n = read(0, buf, sizeof(buf));
      if (n <= 0) {  // parent gone (AppMasterEntryPoint: stdin EOF)
        stdin_open = false;
        m.stop = true;
      }
    }
    std::vector<int> dead;
    for (size_t i = base; i < fds.size(); ++i) {
      if (!(fds[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      Msg q;
      if (!rx_frame::read_msg(fds[i].fd, q)) {
        dead.push_back(fds[i].fd);
        continue;
      }
      Msg rep = m.handle(fds[i].fd, q);
      if (!rx_frame::write_msg(fds[i].fd, rep)) dead.push_back(fds[i].fd);
    }
    for (int d : dead) {
      m.on_disconnected(d);
      m.subscribers.erase(d);
      close(d);
      for (size_t i = 0; i < conns.size(); ++i)
        if (conns[i] == d) {
          conns.erase(conns.begin() + i);
          break;
        }
    }
  }
  m.stop_shuffle_services();
  for (int c : conns) close(c);
  close(m.listen_fd);
  unlink(m.sock_path.c_str());
  return 0;
}
