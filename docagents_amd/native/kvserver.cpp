// docagents native key-value cache: a RESP (Redis protocol) subset, single-threaded epoll.
//
// Replaces the reference's Redis 7 (docker-compose.yml:31-43) for the query-result and
// question-embedding caches (internal/cache/redis.go). Commands: PING, AUTH, ECHO, GET,
// SET key value [EX s | PX ms] [NX | XX], DEL, EXISTS, EXPIRE, TTL, PTTL, SCAN cursor [MATCH p]
// [COUNT n] (full iteration, cursor always 0), KEYS, DBSIZE, FLUSHALL/FLUSHDB, INFO, QUIT.
// TTLs are enforced lazily on access plus a periodic sweep; --maxmemory evicts oldest-expiring
// entries first when the value bytes exceed the budget.
#include <fnmatch.h>

#include <cstdlib>
#include <set>

#include "netloop.h"

using namespace da;

struct Entry {
  std::string val;
  int64_t expire_ms = 0;  // 0 = no expiry
};

struct KV {
  Loop loop;
  std::unordered_map<std::string, Entry> db;
  std::string password;
  std::unordered_map<uint64_t, bool> authed;
  size_t bytes = 0, maxmemory = 0;
  uint64_t hits = 0, misses = 0, cmds = 0;

  void reply_simple(Conn& c, const std::string& s) { loop.send(c, "+" + s + "\r\n"); }
  void reply_err(Conn& c, const std::string& s) { loop.send(c, "-" + s + "\r\n"); }
  void reply_int(Conn& c, long long v) { loop.send(c, ":" + std::to_string(v) + "\r\n"); }
  void reply_bulk(Conn& c, const std::string& s) {
    loop.send(c, "$" + std::to_string(s.size()) + "\r\n");
    loop.send(c, s);
    loop.send(c, "\r\n", 2);
  }
  void reply_nil(Conn& c) { loop.send(c, "$-1\r\n"); }
  void reply_array(Conn& c, const std::vector<std::string>& a) {
    loop.send(c, "*" + std::to_string(a.size()) + "\r\n");
    for (auto& s : a) reply_bulk(c, s);
  }

  Entry* lookup(const std::string& k) {
    auto it = db.find(k);
    if (it == db.end()) return nullptr;
    if (it->second.expire_ms && it->second.expire_ms <= now_ms()) {
      erase(it);
      return nullptr;
    }
    return &it->second;
  }
  void erase(std::unordered_map<std::string, Entry>::iterator it) {
    bytes -= it->first.size() + it->second.val.size();
    db.erase(it);
  }
  void set(const std::string& k, std::string v, int64_t exp) {
    auto it = db.find(k);
    if (it != db.end()) erase(it);
    bytes += k.size() + v.size();
    db[k] = Entry{std::move(v), exp};
    evict();
  }
  void evict() {
    if (!maxmemory || bytes <= maxmemory) return;
    std::vector<std::pair<int64_t, std::string>> order;
    for (auto& kv : db) order.emplace_back(kv.second.expire_ms ? kv.second.expire_ms : INT64_MAX, kv.first);
    std::sort(order.begin(), order.end());
    for (auto& o : order) {
      if (bytes <= maxmemory) break;
      auto it = db.find(o.second);
      if (it != db.end()) erase(it);
    }
  }

  // Limits of the stock server (redis.conf proto-max-bulk-len 512 MB; inline requests 64 KB;
  // multibulk length 1M here): a frame outside them is a protocol error that closes the
  // connection, as Redis does — the rest of the stream cannot be framed.
  static constexpr long kMaxBulk = 512L << 20, kMaxArgs = 1L << 20;
  static constexpr size_t kMaxInline = 64u << 10;

  // strict decimal (optionally negative) between [p, e): false on anything else or overflow
  static bool parse_long(const std::string& in, size_t p, size_t e, long& out) {
    bool neg = p < e && in[p] == '-';
    if (neg) ++p;
    if (p >= e || e - p > 18) return false;
    long v = 0;
    for (size_t i = p; i < e; ++i) {
      if (in[i] < '0' || in[i] > '9') return false;
      v = v * 10 + (in[i] - '0');
    }
    out = neg ? -v : v;
    return true;
  }

  // parse one RESP array command (or inline command): 1 = a command in args, 0 = incomplete,
  // -1 = protocol error (replied; the caller closes the connection)
  int parse(Conn& c, std::vector<std::string>& args) {
    std::string& in = c.in;
    if (in.empty()) return 0;
    if (in[0] != '*') {  // inline
      size_t e = in.find("\r\n");
      if (e == std::string::npos) {
        if (in.size() > kMaxInline) { reply_err(c, "ERR Protocol error: too big inline request"); return -1; }
        return 0;
      }
      if (e > kMaxInline) { reply_err(c, "ERR Protocol error: too big inline request"); return -1; }
      std::string line = in.substr(0, e);
      in.erase(0, e + 2);
      size_t a = 0;
      while (a < line.size()) {
        while (a < line.size() && line[a] == ' ') ++a;
        size_t b = line.find(' ', a);
        if (b == std::string::npos) b = line.size();
        if (b > a) args.push_back(line.substr(a, b - a));
        a = b;
      }
      return 1;
    }
    size_t p = in.find("\r\n");
    if (p == std::string::npos) {
      if (in.size() > kMaxInline) { reply_err(c, "ERR Protocol error: too big multibulk header"); return -1; }
      return 0;
    }
    long n = 0;
    if (!parse_long(in, 1, p, n) || n > kMaxArgs) {
      reply_err(c, "ERR Protocol error: invalid multibulk length");
      return -1;
    }
    size_t pos = p + 2;
    std::vector<std::string> out;
    for (long i = 0; i < n; ++i) {
      if (pos >= in.size()) return 0;
      if (in[pos] != '$') {
        reply_err(c, std::string("ERR Protocol error: expected '$', got '") + in[pos] + "'");
        return -1;
      }
      size_t q = in.find("\r\n", pos);
      if (q == std::string::npos) {
        if (in.size() - pos > kMaxInline) { reply_err(c, "ERR Protocol error: invalid bulk length"); return -1; }
        return 0;
      }
      long len = 0;
      if (!parse_long(in, pos + 1, q, len) || len < 0 || len > kMaxBulk) {
        reply_err(c, "ERR Protocol error: invalid bulk length");
        return -1;
      }
      if (in.size() < q + 2 + (size_t)len + 2) return 0;
      if (in.compare(q + 2 + (size_t)len, 2, "\r\n") != 0) {
        reply_err(c, "ERR Protocol error: bulk not terminated by CRLF");
        return -1;
      }
      out.push_back(in.substr(q + 2, (size_t)len));
      pos = q + 2 + (size_t)len + 2;
    }
    in.erase(0, pos);
    args.swap(out);
    return 1;
  }

  // now + v units, or -1 when that overflows (Redis: "invalid expire time")
  static int64_t expire_at(long long v, int64_t unit_ms) {
    const int64_t t = now_ms();
    if (v <= 0 || v > (INT64_MAX - t) / unit_ms) return -1;
    return t + v * unit_ms;
  }

  static std::string upper(std::string s) {
    for (auto& ch : s) ch = (char)toupper(ch);
    return s;
  }

  void exec(Conn& c, std::vector<std::string>& a) {
    ++cmds;
    if (a.empty()) return;
    std::string cmd = upper(a[0]);
    if (cmd == "AUTH") {
      const std::string& pw = a.back();
      if (password.empty() || pw == password) { authed[c.id] = true; reply_simple(c, "OK"); }
      else reply_err(c, "WRONGPASS invalid username-password pair or user is disabled.");
      return;
    }
    if (!password.empty() && !authed[c.id] && cmd != "PING" && cmd != "QUIT") {
      reply_err(c, "NOAUTH Authentication required.");
      return;
    }
    if (cmd == "PING") { if (a.size() > 1) reply_bulk(c, a[1]); else reply_simple(c, "PONG"); }
    else if (cmd == "ECHO" && a.size() == 2) reply_bulk(c, a[1]);
    else if (cmd == "QUIT") { reply_simple(c, "OK"); loop.close(c); }
    else if (cmd == "GET" && a.size() == 2) {
      Entry* e = lookup(a[1]);
      if (e) { ++hits; reply_bulk(c, e->val); } else { ++misses; reply_nil(c); }
    } else if (cmd == "SET" && a.size() >= 3) {
      int64_t exp = 0;
      bool nx = false, xx = false;
      for (size_t i = 3; i < a.size(); ++i) {
        std::string o = upper(a[i]);
        if ((o == "EX" || o == "PX") && i + 1 < a.size()) {
          exp = expire_at(atoll(a[++i].c_str()), o == "EX" ? 1000 : 1);
          if (exp < 0) { reply_err(c, "ERR invalid expire time in 'set' command"); return; }
        } else if (o == "NX") nx = true;
        else if (o == "XX") xx = true;
        else { reply_err(c, "ERR syntax error"); return; }
      }
      bool exists = lookup(a[1]) != nullptr;
      if ((nx && exists) || (xx && !exists)) { reply_nil(c); return; }
      set(a[1], a[2], exp);
      reply_simple(c, "OK");
    } else if (cmd == "DEL" && a.size() >= 2) {
      long long n = 0;
      for (size_t i = 1; i < a.size(); ++i) {
        auto it = db.find(a[i]);
        if (it != db.end()) { erase(it); ++n; }
      }
      reply_int(c, n);
    } else if (cmd == "EXISTS" && a.size() >= 2) {
      long long n = 0;
      for (size_t i = 1; i < a.size(); ++i) n += lookup(a[i]) != nullptr;
      reply_int(c, n);
    } else if (cmd == "EXPIRE" && a.size() == 3) {
      Entry* e = lookup(a[1]);
      if (!e) { reply_int(c, 0); return; }
      const long long v = atoll(a[2].c_str());
      if (v <= 0) {  // Redis: a non-positive TTL deletes the key
        erase(db.find(a[1]));
        reply_int(c, 1);
        return;
      }
      const int64_t at = expire_at(v, 1000);
      if (at < 0) { reply_err(c, "ERR invalid expire time in 'expire' command"); return; }
      e->expire_ms = at;
      reply_int(c, 1);
    } else if ((cmd == "TTL" || cmd == "PTTL") && a.size() == 2) {
      Entry* e = lookup(a[1]);
      if (!e) reply_int(c, -2);
      else if (!e->expire_ms) reply_int(c, -1);
      else {
        long long ms = e->expire_ms - now_ms();
        reply_int(c, cmd == "TTL" ? (ms + 999) / 1000 : ms);
      }
    } else if (cmd == "SCAN" || cmd == "KEYS") {
      std::string pat = cmd == "KEYS" && a.size() > 1 ? a[1] : "*";
      for (size_t i = 2; i + 1 < a.size(); ++i)
        if (upper(a[i]) == "MATCH") pat = a[i + 1];
      std::vector<std::string> keys;
      int64_t t = now_ms();
      for (auto& kv : db)
        if ((!kv.second.expire_ms || kv.second.expire_ms > t) && fnmatch(pat.c_str(), kv.first.c_str(), 0) == 0)
          keys.push_back(kv.first);
      if (cmd == "KEYS") { reply_array(c, keys); return; }
      loop.send(c, "*2\r\n");
      reply_bulk(c, "0");
      reply_array(c, keys);
    } else if (cmd == "DBSIZE") reply_int(c, (long long)db.size());
    else if (cmd == "FLUSHALL" || cmd == "FLUSHDB") { db.clear(); bytes = 0; reply_simple(c, "OK"); }
    else if (cmd == "INFO") {
      reply_bulk(c, "# Server\r\nredis_version:7.0.0-docagents\r\n# Stats\r\nkeyspace_hits:" + std::to_string(hits) +
                        "\r\nkeyspace_misses:" + std::to_string(misses) + "\r\ntotal_commands_processed:" +
                        std::to_string(cmds) + "\r\n# Memory\r\nused_memory:" + std::to_string(bytes) +
                        "\r\n# Keyspace\r\ndb0:keys=" + std::to_string(db.size()) + "\r\n");
    } else reply_err(c, "ERR unknown command '" + a[0] + "'");
  }

  void sweep() {
    int64_t t = now_ms();
    int budget = 2000;
    for (auto it = db.begin(); it != db.end() && budget > 0; --budget) {
      if (it->second.expire_ms && it->second.expire_ms <= t) {
        bytes -= it->first.size() + it->second.val.size();
        it = db.erase(it);
      } else ++it;
    }
  }
};

int main(int argc, char** argv) {
  std::string addr = "0.0.0.0:6379";
  KV kv;
  for (int i = 1; i < argc; ++i) {
    std::string k = argv[i];
    auto val = [&]() { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
    if (k == "--listen") addr = val();
    else if (k == "--requirepass") kv.password = val();
    else if (k == "--maxmemory") kv.maxmemory = strtoull(val().c_str(), nullptr, 10);
    else if (k == "--help") {
      printf("usage: da-kvserver [--listen host:port] [--requirepass pw] [--maxmemory bytes]\n");
      return 0;
    }
  }
  std::string host;
  int port;
  if (!parse_addr(addr, host, port)) { fprintf(stderr, "bad --listen %s\n", addr.c_str()); return 2; }
  if (!kv.loop.listen_on(host, port)) { perror("listen"); return 1; }
  kv.loop.on_data = [&](Conn& c) {
    std::vector<std::string> a;
    while (true) {
      const int r = kv.parse(c, a);
      if (r < 0) { c.in.clear(); kv.loop.close(c); break; }
      if (r == 0) break;
      kv.exec(c, a);
      a.clear();
      if (c.closing) break;
    }
  };
  kv.loop.on_close = [&](Conn& c) { kv.authed.erase(c.id); };
  kv.loop.on_tick = [&]() { kv.sweep(); };
  fprintf(stderr, "{\"level\":\"INFO\",\"msg\":\"kv cache listening\",\"addr\":\"%s\"}\n", addr.c_str());
  kv.loop.run();
  return 0;
}
