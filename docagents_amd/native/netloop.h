// Minimal single-threaded epoll TCP event loop shared by the native broker and KV cache.
#pragma once
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <stdint.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cstdio>
#include <functional>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

namespace da {

inline int64_t now_ms() {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  return (int64_t)tv.tv_sec * 1000 + tv.tv_usec / 1000;
}

struct Conn {
  int fd = -1;
  uint64_t id = 0;
  std::string in;      // unparsed input
  std::string out;     // pending output
  bool closing = false;
  void* user = nullptr;
};

class Loop {
 public:
  std::function<void(Conn&)> on_open;
  std::function<void(Conn&)> on_data;   // consume from c.in
  std::function<void(Conn&)> on_close;
  std::function<void()> on_tick;        // every ~100 ms

  bool listen_on(const std::string& host, int port) {
    lfd_ = socket(AF_INET, SOCK_STREAM, 0);
    if (lfd_ < 0) return false;
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    if (host.empty() || host == "0.0.0.0") a.sin_addr.s_addr = INADDR_ANY;
    else if (inet_pton(AF_INET, host == "localhost" ? "127.0.0.1" : host.c_str(), &a.sin_addr) != 1) return false;
    if (bind(lfd_, (sockaddr*)&a, sizeof a) < 0) return false;
    if (listen(lfd_, 512) < 0) return false;
    nonblock(lfd_);
    ep_ = epoll_create1(0);
    add(lfd_, EPOLLIN);
    return true;
  }

  void send(Conn& c, const char* p, size_t n) {
    c.out.append(p, n);
    dirty_.push_back(c.id);
  }
  void send(Conn& c, const std::string& s) { send(c, s.data(), s.size()); }
  void close(Conn& c) { c.closing = true; dirty_.push_back(c.id); }
  Conn* get(uint64_t id) {
    auto it = conns_.find(id);
    return it == conns_.end() ? nullptr : it->second.get();
  }
  size_t nconns() const { return conns_.size(); }

  void run() {
    signal(SIGPIPE, SIG_IGN);
    std::vector<epoll_event> evs(256);
    int64_t last_tick = now_ms();
    while (!stop_) {
      int n = epoll_wait(ep_, evs.data(), (int)evs.size(), 50);
      for (int i = 0; i < n; ++i) {
        if (evs[i].data.u64 == 0) { accept_all(); continue; }
        Conn* c = get(evs[i].data.u64);
        if (!c) continue;
        if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) read_conn(*c);
        if (c && (evs[i].events & EPOLLOUT)) dirty_.push_back(c->id);
      }
      flush_dirty();
      int64_t t = now_ms();
      if (t - last_tick >= 100) {
        last_tick = t;
        if (on_tick) on_tick();
        flush_dirty();
      }
    }
  }
  void stop() { stop_ = true; }

 private:
  int lfd_ = -1, ep_ = -1;
  uint64_t next_id_ = 1;
  bool stop_ = false;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns_;
  std::vector<uint64_t> dirty_;

  static void nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }
  void add(int fd, uint32_t ev, uint64_t id = 0) {
    epoll_event e{};
    e.events = ev;
    e.data.u64 = id;
    epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e);
  }
  void mod(int fd, uint32_t ev, uint64_t id) {
    epoll_event e{};
    e.events = ev;
    e.data.u64 = id;
    epoll_ctl(ep_, EPOLL_CTL_MOD, fd, &e);
  }
  void accept_all() {
    while (true) {
      int fd = accept(lfd_, nullptr, nullptr);
      if (fd < 0) return;
      nonblock(fd);
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      c->id = next_id_++;
      Conn* raw = c.get();
      conns_[raw->id] = std::move(c);
      add(fd, EPOLLIN, raw->id);
      if (on_open) on_open(*raw);
    }
  }
  void read_conn(Conn& c) {
    char buf[65536];
    while (true) {
      ssize_t r = ::read(c.fd, buf, sizeof buf);
      if (r > 0) { c.in.append(buf, (size_t)r); continue; }
      if (r == 0) { c.closing = true; break; }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      if (errno == EINTR) continue;
      c.closing = true;
      break;
    }
    if (!c.in.empty() && on_data) on_data(c);
    dirty_.push_back(c.id);
  }
  void flush_dirty() {
    while (!dirty_.empty()) {
      std::vector<uint64_t> ids;
      ids.swap(dirty_);
      for (uint64_t id : ids) {
        Conn* c = get(id);
        if (!c) continue;
        while (!c->out.empty()) {
          ssize_t w = ::write(c->fd, c->out.data(), c->out.size());
          if (w > 0) { c->out.erase(0, (size_t)w); continue; }
          if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
          if (w < 0 && errno == EINTR) continue;
          c->closing = true;
          c->out.clear();
          break;
        }
        if (c->closing && (c->out.empty())) {
          if (on_close) on_close(*c);
          epoll_ctl(ep_, EPOLL_CTL_DEL, c->fd, nullptr);
          ::close(c->fd);
          conns_.erase(id);
          continue;
        }
        mod(c->fd, c->out.empty() ? EPOLLIN : (EPOLLIN | EPOLLOUT), id);
      }
    }
  }
};

inline bool parse_addr(const std::string& s, std::string& host, int& port) {
  std::string x = s;
  auto p = x.find("://");
  if (p != std::string::npos) x = x.substr(p + 3);
  auto c = x.rfind(':');
  if (c == std::string::npos) return false;
  host = x.substr(0, c);
  port = atoi(x.c_str() + c + 1);
  return port > 0;
}

}  // namespace da
