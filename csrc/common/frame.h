// Length-prefixed string-list frames over Unix-domain sockets: the wire format of every native
// control service (actor supervisor, app master, shuffle service).
//
//   frame   = u32 payload_len | payload
//   payload = u32 op | u32 nstr | nstr x (u32 len | bytes)
//
// An optional file descriptor rides along a frame as SCM_RIGHTS ancillary data (the shuffle
// service hands out map-output files that way, so a reducer mmaps them instead of copying).
#pragma once
#include <errno.h>
#include <stdint.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <string>
#include <vector>

namespace rx_frame {

struct Msg {
  uint32_t op = 0;
  std::vector<std::string> s;
};

inline bool write_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    c += w;
    n -= (size_t)w;
  }
  return true;
}

inline bool read_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t r = ::recv(fd, c, n, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    c += r;
    n -= (size_t)r;
  }
  return true;
}

inline std::string encode(const Msg& m) {
  std::string out(12, '\0');
  uint32_t n = (uint32_t)m.s.size();
  memcpy(&out[4], &m.op, 4);
  memcpy(&out[8], &n, 4);
  for (const std::string& x : m.s) {
    uint32_t l = (uint32_t)x.size();
    out.append((const char*)&l, 4);
    out.append(x);
  }
  uint32_t len = (uint32_t)(out.size() - 4);
  memcpy(&out[0], &len, 4);
  return out;
}

inline bool decode(const std::string& payload, Msg& m) {
  if (payload.size() < 8) return false;
  uint32_t n;
  memcpy(&m.op, payload.data(), 4);
  memcpy(&n, payload.data() + 4, 4);
  size_t off = 8;
  m.s.clear();
  for (uint32_t i = 0; i < n; ++i) {
    if (off + 4 > payload.size()) return false;
    uint32_t l;
    memcpy(&l, payload.data() + off, 4);
    off += 4;
    if (off + l > payload.size()) return false;
    m.s.emplace_back(payload.data() + off, l);
    off += l;
  }
  return true;
}

inline bool write_msg(int fd, const Msg& m) {
  const std::string b = encode(m);
  return write_all(fd, b.data(), b.size());
}

// Frame plus one descriptor (SCM_RIGHTS) attached to its first byte.
inline bool write_msg_fd(int fd, const Msg& m, int pass_fd) {
  const std::string b = encode(m);
  struct iovec iov = {(void*)b.data(), 1};
  char ctl[CMSG_SPACE(sizeof(int))];
  memset(ctl, 0, sizeof(ctl));
  struct msghdr h;
  memset(&h, 0, sizeof(h));
  h.msg_iov = &iov;
  h.msg_iovlen = 1;
  h.msg_control = ctl;
  h.msg_controllen = sizeof(ctl);
  struct cmsghdr* c = CMSG_FIRSTHDR(&h);
  c->cmsg_level = SOL_SOCKET;
  c->cmsg_type = SCM_RIGHTS;
  c->cmsg_len = CMSG_LEN(sizeof(int));
  memcpy(CMSG_DATA(c), &pass_fd, sizeof(int));
  ssize_t w;
  do {
    w = ::sendmsg(fd, &h, MSG_NOSIGNAL);
  } while (w < 0 && errno == EINTR);
  if (w != 1) return false;
  return write_all(fd, b.data() + 1, b.size() - 1);
}

// Returns false on EOF / error. Payload sizes above `cap` are refused.
inline bool read_msg(int fd, Msg& m, size_t cap = 64u << 20) {
  uint32_t len;
  if (!read_all(fd, &len, 4)) return false;
  if (len > cap) return false;
  std::string payload(len, '\0');
  if (len && !read_all(fd, &payload[0], len)) return false;
  return decode(payload, m);
}

inline int listen_unix(const std::string& path, int backlog = 128) {
  int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  struct sockaddr_un a;
  memset(&a, 0, sizeof(a));
  a.sun_family = AF_UNIX;
  if (path.size() >= sizeof(a.sun_path)) {
    ::close(fd);
    return -1;
  }
  strncpy(a.sun_path, path.c_str(), sizeof(a.sun_path) - 1);
  ::unlink(path.c_str());
  if (::bind(fd, (struct sockaddr*)&a, sizeof(a)) < 0 || ::listen(fd, backlog) < 0) {
    ::close(fd);
    return -1;
  }
  return fd;
}

}  // namespace rx_frame
