// docagents native message broker: a NATS core protocol subset (single-threaded epoll).
//
// Replaces the reference's nats-server (docker-compose.yml:18-29). Wire-compatible with NATS
// core clients for: INFO, CONNECT, PUB, SUB (with queue group), UNSUB, PING/PONG, MSG, +OK, -ERR,
// with `*` / `>` subject wildcards and round-robin queue-group delivery (the reference's
// `QueueSubscribe(subject, "workers-"+type)`, internal/queue/nats.go:40-51).
//
// Extensions for at-least-once task delivery (the reference is at-most-once, README.md:717-722):
//  * durable subjects (prefix "tasks." by default): a message published while no subscriber
//    matches is buffered and delivered when one subscribes (instead of being dropped);
//  * queue-group deliveries on durable subjects carry a reply subject "$ACK.<seq>"; the worker
//    publishes (empty) to it when done. Unacked messages are redelivered when the consumer's
//    connection drops or after --ack-wait seconds, up to --max-deliver times, then published to
//    "$DLQ.<subject>" (dead-letter subject) and dropped.
//  * "$SYS.REQ.STATS" request -> JSON counters on the reply subject.
#include <algorithm>
#include <cstdlib>
#include <deque>
#include <map>
#include <sstream>
#include <unordered_set>

#include "netloop.h"

using namespace da;

struct Sub {
  uint64_t conn;
  std::string sid, subject, queue;
  std::vector<std::string> toks;
  long max_msgs = -1, got = 0;
};

struct Pending {  // unacked durable delivery
  std::string subject, data;
  uint64_t conn;
  int64_t deadline;
  int deliveries;
};

static std::vector<std::string> split_tokens(const std::string& s, char sep) {
  std::vector<std::string> out;
  size_t a = 0;
  while (true) {
    size_t b = s.find(sep, a);
    out.push_back(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
    if (b == std::string::npos) break;
    a = b + 1;
  }
  return out;
}

static bool match(const std::vector<std::string>& pat, const std::vector<std::string>& sub) {
  size_t i = 0;
  for (; i < pat.size(); ++i) {
    if (pat[i] == ">") return sub.size() > i;
    if (i >= sub.size()) return false;
    if (pat[i] != "*" && pat[i] != sub[i]) return false;
  }
  return i == sub.size();
}

struct Broker {
  Loop loop;
  std::map<std::pair<uint64_t, std::string>, Sub> subs;   // (conn, sid) -> sub
  std::map<std::string, uint64_t> rr;                     // queue group round robin
  std::deque<std::pair<std::string, std::string>> parked; // durable msgs with no subscriber
  std::map<uint64_t, Pending> unacked;
  uint64_t ack_seq = 1;
  std::string durable_prefix = "tasks.";
  int ack_wait_ms = 300000, max_deliver = 5;
  size_t max_parked = 1000000;
  size_t max_payload = 64u << 20;  // advertised in INFO
  uint64_t n_pub = 0, n_msg = 0, n_redeliver = 0, n_dlq = 0, n_acks = 0;
  std::unordered_map<uint64_t, bool> verbose;

  bool durable(const std::string& s) const {
    return !durable_prefix.empty() && s.compare(0, durable_prefix.size(), durable_prefix) == 0;
  }

  void send_msg(Conn& c, const std::string& subject, const std::string& sid, const std::string& reply,
                const std::string& data) {
    std::string h = "MSG " + subject + " " + sid + " ";
    if (!reply.empty()) h += reply + " ";
    h += std::to_string(data.size()) + "\r\n";
    loop.send(c, h);
    loop.send(c, data);
    loop.send(c, "\r\n", 2);
    ++n_msg;
  }

  // returns number of deliveries
  int route(const std::string& subject, const std::string& reply, const std::string& data, int deliveries = 0) {
    auto toks = split_tokens(subject, '.');
    std::map<std::string, std::vector<Sub*>> groups;
    int delivered = 0;
    for (auto& kv : subs) {
      Sub& s = kv.second;
      if (!match(s.toks, toks)) continue;
      if (s.queue.empty()) {
        Conn* c = loop.get(s.conn);
        if (!c) continue;
        send_msg(*c, subject, s.sid, reply, data);
        ++delivered;
        bump(s);
      } else {
        groups[s.queue].push_back(&s);
      }
    }
    for (auto& g : groups) {
      auto& members = g.second;
      uint64_t k = rr[subject + "|" + g.first]++;
      Sub* s = members[k % members.size()];
      Conn* c = loop.get(s->conn);
      if (!c) continue;
      std::string rep = reply;
      if (durable(subject) && reply.empty()) {
        uint64_t id = ack_seq++;
        rep = "$ACK." + std::to_string(id);
        unacked[id] = Pending{subject, data, s->conn, now_ms() + ack_wait_ms, deliveries + 1};
      }
      send_msg(*c, subject, s->sid, rep, data);
      ++delivered;
      bump(*s);
    }
    return delivered;
  }

  void bump(Sub& s) {
    if (s.max_msgs > 0 && ++s.got >= s.max_msgs) s.max_msgs = 0;  // auto-unsub lazily
  }

  void publish(const std::string& subject, const std::string& reply, const std::string& data) {
    ++n_pub;
    if (subject.compare(0, 5, "$ACK.") == 0) {
      uint64_t id = strtoull(subject.c_str() + 5, nullptr, 10);
      if (unacked.erase(id)) ++n_acks;
      return;
    }
    if (subject == "$SYS.REQ.STATS" && !reply.empty()) {
      std::ostringstream o;
      o << "{\"conns\":" << loop.nconns() << ",\"subs\":" << subs.size() << ",\"published\":" << n_pub
        << ",\"delivered\":" << n_msg << ",\"parked\":" << parked.size() << ",\"unacked\":" << unacked.size()
        << ",\"redelivered\":" << n_redeliver << ",\"dead_lettered\":" << n_dlq << ",\"acks\":" << n_acks << "}";
      route(reply, "", o.str());
      return;
    }
    int d = route(subject, reply, data);
    if (d == 0 && durable(subject) && parked.size() < max_parked) parked.emplace_back(subject, data);
  }

  void redeliver(uint64_t id) {
    auto it = unacked.find(id);
    if (it == unacked.end()) return;
    Pending p = it->second;
    unacked.erase(it);
    if (p.deliveries >= max_deliver) {
      ++n_dlq;
      route("$DLQ." + p.subject, "", p.data);
      return;
    }
    ++n_redeliver;
    if (route(p.subject, "", p.data, p.deliveries) == 0) parked.emplace_back(p.subject, p.data);
  }

  void flush_parked() {
    if (parked.empty()) return;
    std::deque<std::pair<std::string, std::string>> keep;
    while (!parked.empty()) {
      auto m = std::move(parked.front());
      parked.pop_front();
      if (route(m.first, "", m.second) == 0) keep.push_back(std::move(m));
    }
    parked.swap(keep);
  }

  void err(Conn& c, const std::string& m) { loop.send(c, "-ERR '" + m + "'\r\n"); }

  void handle(Conn& c) {
    while (true) {
      size_t e = c.in.find("\r\n");
      if (e == std::string::npos) {
        if (c.in.size() > (1u << 20)) { err(c, "Maximum Control Line Exceeded"); c.in.clear(); loop.close(c); }
        return;
      }
      if (e > (1u << 20)) { err(c, "Maximum Control Line Exceeded"); c.in.clear(); loop.close(c); return; }
      std::string line = c.in.substr(0, e);
      std::string verb = line.substr(0, line.find(' '));
      std::transform(verb.begin(), verb.end(), verb.begin(), ::toupper);
      std::vector<std::string> a;
      {
        std::istringstream is(line);
        std::string t;
        while (is >> t) a.push_back(t);
      }
      if (verb == "PUB") {
        if (a.size() < 3 || a.size() > 4) { err(c, "Unknown Protocol Operation"); c.in.erase(0, e + 2); continue; }
        // the size must be a plain decimal within max_payload (nats-server: "Maximum Payload
        // Violation", then the connection is closed: the rest of the stream cannot be framed)
        const std::string& ns = a.back();
        size_t n = 0;
        bool ok = !ns.empty() && ns.size() <= 10;
        for (char ch : ns) ok = ok && ch >= '0' && ch <= '9';
        if (ok) n = strtoull(ns.c_str(), nullptr, 10);
        if (!ok || n > max_payload) {
          err(c, ok ? "Maximum Payload Violation" : "Invalid Message Size");
          c.in.clear();
          loop.close(c);
          return;
        }
        if (c.in.size() < e + 2 + n + 2) return;  // wait for payload
        std::string data = c.in.substr(e + 2, n);
        c.in.erase(0, e + 2 + n + 2);
        publish(a[1], a.size() == 4 ? a[2] : "", data);
        if (verbose[c.id]) loop.send(c, "+OK\r\n");
        continue;
      }
      c.in.erase(0, e + 2);
      if (verb == "PING") {
        loop.send(c, "PONG\r\n");
      } else if (verb == "PONG") {
      } else if (verb == "CONNECT") {
        verbose[c.id] = line.find("\"verbose\":true") != std::string::npos;
        if (verbose[c.id]) loop.send(c, "+OK\r\n");
      } else if (verb == "SUB") {
        if (a.size() < 3) { err(c, "Unknown Protocol Operation"); continue; }
        Sub s;
        s.conn = c.id;
        s.subject = a[1];
        s.queue = a.size() == 4 ? a[2] : "";
        s.sid = a.back();
        s.toks = split_tokens(s.subject, '.');
        subs[{c.id, s.sid}] = s;
        if (verbose[c.id]) loop.send(c, "+OK\r\n");
        flush_parked();
      } else if (verb == "UNSUB") {
        if (a.size() < 2) { err(c, "Unknown Protocol Operation"); continue; }
        auto it = subs.find({c.id, a[1]});
        if (it != subs.end()) {
          if (a.size() == 3) it->second.max_msgs = atol(a[2].c_str());
          else subs.erase(it);
        }
        if (verbose[c.id]) loop.send(c, "+OK\r\n");
      } else {
        err(c, "Unknown Protocol Operation");
      }
    }
  }

  void on_close(Conn& c) {
    for (auto it = subs.begin(); it != subs.end();) {
      if (it->first.first == c.id) it = subs.erase(it);
      else ++it;
    }
    std::vector<uint64_t> lost;
    for (auto& kv : unacked)
      if (kv.second.conn == c.id) lost.push_back(kv.first);
    for (uint64_t id : lost) redeliver(id);
    verbose.erase(c.id);
  }

  void tick() {
    for (auto it = subs.begin(); it != subs.end();) {  // expired auto-unsubs
      if (it->second.max_msgs == 0) it = subs.erase(it);
      else ++it;
    }
    int64_t t = now_ms();
    std::vector<uint64_t> late;
    for (auto& kv : unacked)
      if (kv.second.deadline <= t) late.push_back(kv.first);
    for (uint64_t id : late) redeliver(id);
    flush_parked();
  }
};

int main(int argc, char** argv) {
  std::string addr = "0.0.0.0:4222";
  Broker b;
  for (int i = 1; i < argc; ++i) {
    std::string k = argv[i];
    auto val = [&]() { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
    if (k == "--listen") addr = val();
    else if (k == "--ack-wait") b.ack_wait_ms = (int)(atof(val().c_str()) * 1000);
    else if (k == "--max-deliver") b.max_deliver = atoi(val().c_str());
    else if (k == "--durable-prefix") b.durable_prefix = val();
    else if (k == "--help") {
      printf("usage: da-broker [--listen host:port] [--ack-wait s] [--max-deliver n] [--durable-prefix p]\n");
      return 0;
    }
  }
  std::string host;
  int port;
  if (!parse_addr(addr, host, port)) { fprintf(stderr, "bad --listen %s\n", addr.c_str()); return 2; }
  if (!b.loop.listen_on(host, port)) { perror("listen"); return 1; }
  b.loop.on_open = [&](Conn& c) {
    std::string info = "INFO {\"server_id\":\"docagents-broker\",\"server_name\":\"docagents-broker\",\"version\":\"2.10.0\","
                       "\"proto\":1,\"go\":\"none\",\"host\":\"" + host + "\",\"port\":" + std::to_string(port) +
                       ",\"headers\":false,\"max_payload\":67108864}\r\n";
    b.loop.send(c, info);
  };
  b.loop.on_data = [&](Conn& c) { b.handle(c); };
  b.loop.on_close = [&](Conn& c) { b.on_close(c); };
  b.loop.on_tick = [&]() { b.tick(); };
  fprintf(stderr, "{\"level\":\"INFO\",\"msg\":\"broker listening\",\"addr\":\"%s\"}\n", addr.c_str());
  b.loop.run();
  return 0;
}
