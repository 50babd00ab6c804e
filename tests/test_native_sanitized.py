"""The native replacements of nats-server and redis (docker-compose.yml:18-43) built with
AddressSanitizer + UndefinedBehaviorSanitizer (host code; -fno-sanitize-recover: the first finding
aborts the server) and fed malformed, partial (byte-by-byte), pipelined, oversized and random
protocol frames. After every case the server must still be alive and answer a fresh connection;
at the end its stderr must hold no sanitizer report. Plus a differential fuzz of the native chunker
under the same sanitizers (tests/native_fuzz/textfast_fuzz.cpp)."""
import os
import random
import socket
import subprocess
import time

import pytest

from docagents_amd.native import build_sanitized

HERE = os.path.dirname(os.path.abspath(__file__))
SAN_ENV = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def bins(tmp_path_factory):
    return build_sanitized(tmp_path_factory.mktemp("san"),
                           {"textfast_fuzz": [os.path.join(HERE, "native_fuzz", "textfast_fuzz.cpp")]})


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Server:
    def __init__(self, exe, args, tmp):
        self.port = _port()
        self.err_path = tmp / (os.path.basename(str(exe)) + ".stderr")
        self.err = open(self.err_path, "wb")
        self.p = subprocess.Popen([str(exe), "--listen", f"127.0.0.1:{self.port}", *args], stderr=self.err,
                                  env=SAN_ENV)
        t0 = time.time()
        while time.time() - t0 < 20:
            try:
                socket.create_connection(("127.0.0.1", self.port), 0.2).close()
                return
            except OSError:
                time.sleep(0.05)
        raise TimeoutError("server did not start")

    def conn(self):
        s = socket.create_connection(("127.0.0.1", self.port), 5)
        s.settimeout(5)
        return s

    def alive(self):
        return self.p.poll() is None

    def stop(self):
        self.p.kill()
        self.p.wait()
        self.err.close()
        return self.err_path.read_text(errors="replace")


def _recv_until(s, token: bytes, limit=1 << 22):
    buf = b""
    while token not in buf and len(buf) < limit:
        try:
            b = s.recv(65536)
        except socket.timeout:
            break
        if not b:
            break
        buf += b
    return buf


def _drain(s, wait=0.15):
    s.settimeout(wait)
    out = b""
    try:
        while True:
            b = s.recv(65536)
            if not b:
                break
            out += b
    except (socket.timeout, ConnectionError):
        pass
    return out


def _clean(report: str):
    assert "AddressSanitizer" not in report and "runtime error" not in report and "LeakSanitizer" not in report, \
        report[-3000:]


# ----------------------------------------------------------------------------------- broker
def _nats_ok(srv):
    s = srv.conn()
    _recv_until(s, b"\r\n")  # INFO
    s.sendall(b"CONNECT {}\r\nPING\r\n")
    ok = b"PONG" in _recv_until(s, b"PONG")
    s.close()
    return ok


BROKER_BAD = [
    b"PUB\r\n", b"PUB foo\r\n", b"PUB foo -5\r\nxx\r\n", b"PUB foo 99999999999999999999\r\n",
    b"PUB foo abc\r\nabc\r\n", b"PUB foo bar baz qux 3\r\nabc\r\n", b"PUB foo 104857600\r\n",
    b"SUB\r\n", b"SUB x\r\n", b"UNSUB\r\n", b"UNSUB 1 notnum\r\n", b"\r\n\r\n\r\n", b"XYZ junk\r\n",
    b"CONNECT {garbage\r\n", b"\x00\xff\xfe\r\n", b"PUB tasks.parse 3\r\nabcXY", b"sub a.>.b q 1\r\n",
    b"PUB $ACK.18446744073709551616 0\r\n\r\n", b"PUB $SYS.REQ.STATS _INBOX.x 0\r\n\r\n",
]


def test_broker_survives_malformed_partial_pipelined_and_random_frames(bins, tmp_path):
    srv = Server(bins["da-broker"], ["--ack-wait", "1", "--max-deliver", "2"], tmp_path)
    try:
        # byte-by-byte valid session
        s = srv.conn()
        _recv_until(s, b"\r\n")
        for ch in b"CONNECT {}\r\nSUB foo 1\r\nPUB foo 5\r\nhello\r\nPING\r\n":
            s.sendall(bytes([ch]))
        got = _recv_until(s, b"PONG")
        assert b"MSG foo 1 5\r\nhello\r\n" in got, got
        # pipelined: 2000 publishes in one write
        s.sendall(b"".join(b"PUB foo 3\r\nabc\r\n" for _ in range(2000)) + b"PING\r\n")
        got = _recv_until(s, b"PONG")
        assert got.count(b"MSG foo 1 3") == 2000, got.count(b"MSG foo 1 3")
        s.close()
        # malformed frames, each on its own connection
        for bad in BROKER_BAD:
            c = srv.conn()
            _recv_until(c, b"\r\n")
            c.sendall(bad)
            _drain(c)
            c.close()
            assert srv.alive() and _nats_ok(srv), bad
        # oversized control line and oversized declared payload: -ERR and the connection closes
        c = srv.conn()
        _recv_until(c, b"\r\n")
        c.sendall(b"PUB " + b"x" * (2 << 20))
        assert b"Maximum Control Line Exceeded" in _drain(c, 1.0)
        c.close()
        c = srv.conn()
        _recv_until(c, b"\r\n")
        c.sendall(b"PUB big 104857600\r\n")
        assert b"Maximum Payload Violation" in _drain(c, 1.0)
        c.close()
        # durable message delivered, consumer vanishes unacked -> redelivery / DLQ paths
        w = srv.conn()
        _recv_until(w, b"\r\n")
        w.sendall(b"CONNECT {}\r\nSUB tasks.x workers 1\r\nPUB tasks.x 2\r\nhi\r\nPING\r\n")
        _recv_until(w, b"PONG")
        w.close()
        # random frames assembled from protocol fragments and random bytes
        rng = random.Random(7)
        frag = [b"PUB ", b"SUB ", b"UNSUB ", b"PING", b"PONG", b"CONNECT ", b"MSG ", b"foo", b"tasks.a", b" ",
                b"\r\n", b"5", b"-1", b"99999", b"q", b"*", b">", b"$ACK.", b"\x00", b"\xff"]
        for i in range(150):
            c = srv.conn()
            _recv_until(c, b"\r\n")
            data = b"".join(rng.choice(frag) if rng.random() < 0.8 else bytes([rng.randrange(256)])
                            for _ in range(rng.randrange(1, 60)))
            if rng.random() < 0.5:
                for j in range(0, len(data), 3):
                    c.sendall(data[j:j + 3])
            else:
                c.sendall(data)
            _drain(c, 0.02)
            c.close()
        time.sleep(1.5)  # ack-wait ticks run over the parked / unacked state left behind
        assert srv.alive() and _nats_ok(srv)
    finally:
        report = srv.stop()
    _clean(report)


# ----------------------------------------------------------------------------------- kv
def _resp(*args):
    out = b"*%d\r\n" % len(args)
    for a in args:
        a = a if isinstance(a, bytes) else str(a).encode()
        out += b"$%d\r\n%s\r\n" % (len(a), a)
    return out


def _kv_ok(srv):
    s = srv.conn()
    s.sendall(_resp("AUTH", "pw") + _resp("PING"))
    ok = b"+PONG" in _recv_until(s, b"PONG")
    s.close()
    return ok


KV_BAD = [
    b"*-5\r\n", b"*99999999999\r\n", b"*1\r\n$-3\r\nabc\r\n", b"*1\r\n$999999999999\r\n",
    b"*2\r\n$3\r\nGET\r\n:5\r\n", b"*1\r\n$3\r\nGETxx", b"*x\r\n", b"*1\r\n$abc\r\n", b"*1\r\n$\r\n\r\n",
    _resp("SET", "k", "v", "EX", "9223372036854775807"), _resp("SET", "k", "v", "PX", "-1"),
    _resp("SET", "k", "v", "EX", "notanumber"), _resp("SET", "k", "v", "NX", "XX", "EX"),
    _resp("EXPIRE", "k", "9223372036854775807"), _resp("EXPIRE", "k", "-9223372036854775807"),
    _resp("AUTH"), _resp("GET"), _resp("SCAN", "0", "MATCH", "[[[[" * 50), _resp(""),
    b"\r\n", b"   \r\n", b"GET\r\n", b"\x00\x01\x02\r\n",
]


def test_kvserver_survives_malformed_partial_pipelined_and_random_frames(bins, tmp_path):
    srv = Server(bins["da-kvserver"], ["--requirepass", "pw", "--maxmemory", "100000"], tmp_path)
    try:
        s = srv.conn()
        for ch in _resp("AUTH", "pw") + _resp("SET", "k", "hello", "EX", "100") + _resp("GET", "k"):
            s.sendall(bytes([ch]))
        got = _recv_until(s, b"hello")
        assert b"$5\r\nhello\r\n" in got, got
        s.sendall(b"".join(_resp("SET", f"p{i}", "v" * 10) + _resp("GET", f"p{i}") for i in range(2000))
                  + _resp("ECHO", "end"))
        got = _recv_until(s, b"$3\r\nend")
        assert got.count(b"+OK") == 2000 and got.count(b"$10\r\n") == 2000
        s.close()
        for bad in KV_BAD:
            c = srv.conn()
            c.sendall(_resp("AUTH", "pw") + bad)
            _drain(c)
            c.close()
            assert srv.alive() and _kv_ok(srv), bad
        # oversized inline request and oversized bulk declaration: protocol error, connection closed
        for big in (b"x" * (100 << 10), b"*1\r\n$536870913\r\n"):
            c = srv.conn()
            c.sendall(big)
            assert b"Protocol error" in _drain(c, 1.0)
            c.close()
        # an expire overflow must be refused, not wrap into the past
        c = srv.conn()
        c.sendall(_resp("AUTH", "pw") + _resp("SET", "ttl", "v", "EX", "9223372036854775") + _resp("GET", "ttl"))
        got = _drain(c, 0.5)
        assert b"invalid expire time" in got and b"$-1" in got, got
        c.close()
        rng = random.Random(11)
        frag = [b"*", b"$", b"\r\n", b"1", b"2", b"3", b"-1", b"999999", b"GET", b"SET", b"EX", b"k", b"AUTH",
                b"pw", b" ", b"DEL", b"SCAN", b"MATCH", b"\x00"]
        for i in range(200):
            c = srv.conn()
            data = b"".join(rng.choice(frag) if rng.random() < 0.8 else bytes([rng.randrange(256)])
                            for _ in range(rng.randrange(1, 50)))
            c.sendall(_resp("AUTH", "pw"))
            if rng.random() < 0.5:
                for j in range(0, len(data), 2):
                    c.sendall(data[j:j + 2])
            else:
                c.sendall(data)
            _drain(c, 0.02)
            c.close()
        assert srv.alive() and _kv_ok(srv)
    finally:
        report = srv.stop()
    _clean(report)


def test_chunker_differential_fuzz_under_sanitizers(bins):
    r = subprocess.run([str(bins["textfast_fuzz"]), "20000"], capture_output=True, text=True, env=SAN_ENV, timeout=300)
    assert r.returncode == 0, (r.stdout, r.stderr[-3000:])
    assert '"mismatches": 0' in r.stdout
    _clean(r.stderr)
