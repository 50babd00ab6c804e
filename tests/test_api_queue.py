"""Wire formats (Go JSON, errors, validation messages, task envelope), multipart/PDF parsing and
the queue semantics (EnqueueWithRetry, queue groups, NotBefore retry, permanent failure)."""
import asyncio
import base64
import datetime as dt
import json

import pytest

from docagents_amd.api import gojson
from docagents_amd.api.http import fail, write_json
from docagents_amd.api.validation import PayloadError, decode_query_request, validate_query_request
from docagents_amd.queue import inproc as inproc_mod
from docagents_amd.queue.inproc import InProcBus, InProcQueue
from docagents_amd.queue.task import Task, enqueue_with_retry, next_retry
from docagents_amd.text import multipart
from docagents_amd.text.pdf import extract_text, make_pdf
from docagents_amd.utils.log import discard

U1 = "3f1c2b7e-8d4a-4c1e-9f0a-1b2c3d4e5f60"


def test_go_json_writer():
    body = gojson.dumps({"summary": "s", "key_points": ["a", "b"]})
    assert body == '{\n  "key_points": [\n    "a",\n    "b"\n  ],\n  "summary": "s"\n}\n'
    assert gojson.dumps({"x": gojson.F32(0.95)}) == '{\n  "x": 0.95\n}\n'
    assert gojson.dumps({"x": gojson.F32(0.1 + 0.2)}) == '{\n  "x": 0.3\n}\n'
    assert gojson.dumps({"x": None, "y": []}) == '{\n  "x": null,\n  "y": []\n}\n'


def test_error_body_is_plain_text():
    r = fail(None, "invalid payload", None, 400)
    assert r.status_code == 400 and r.body == b"invalid payload\n"
    assert r.headers["content-type"] == "text/plain; charset=utf-8"
    assert r.headers["x-content-type-options"] == "nosniff"
    ok = write_json(202, {"document_id": "x", "status": "processing"})
    assert ok.headers["content-type"] == "application/json"


@pytest.mark.parametrize("body,msgs", [
    ({"question": "", "document_ids": [U1]}, ["Question is required"]),
    ({"question": "Hi", "document_ids": [U1]}, ["Question must be at least 3"]),
    ({"question": "x" * 501, "document_ids": [U1]}, ["Question must be at most 500"]),
    ({"question": "Valid question here", "document_ids": ["not-a-uuid"]}, ["DocumentIDs[0] must be a valid UUID"]),
    ({"question": "Valid question", "document_ids": []}, ["DocumentIDs must be at least 1"]),
    ({"question": "Valid question"}, ["DocumentIDs is required"]),
    ({"question": "Valid question", "document_ids": [U1], "top_k": 25}, ["TopK must be at most 20"]),
    ({"question": "Valid question", "document_ids": [U1], "top_k": -1}, ["TopK must be at least 1"]),
    ({"question": "", "document_ids": []}, ["Question is required", "DocumentIDs must be at least 1"]),
    ({"question": "Valid question", "document_ids": [U1.upper()]}, ["DocumentIDs[0] must be a valid UUID"]),
    ({"question": "Valid question", "document_ids": [U1], "top_k": 0}, []),
])
def test_validation_messages(body, msgs):
    req = decode_query_request(json.dumps(body).encode())
    assert validate_query_request(req) == msgs


def test_decode_errors():
    for bad in (b"{invalid json}", b'{"question": 5}', b'{"top_k": 2.5}', b'{"document_ids": "x"}', b"[1]"):
        with pytest.raises(PayloadError):
            decode_query_request(bad)
    r = decode_query_request(b'{"Question": "abc", "DOCUMENT_IDS": ["%s"]} trailing' % U1.encode())
    assert r.question == "abc" and r.document_ids == [U1]  # case-insensitive keys, one value decoded


def test_task_envelope_wire_format():
    t = Task(type="parse", payload=b'{"a":1}', id="11111111-1111-4111-8111-111111111111")
    d = json.loads(t.encode())
    assert set(d) == {"ID", "Type", "Payload", "Attempts", "MaxAttempts", "NotBefore"}
    assert base64.b64decode(d["Payload"]) == b'{"a":1}' and d["NotBefore"] == "0001-01-01T00:00:00Z"
    go = b'{"ID":"x","Type":"analyze","Payload":"eyJiIjoyfQ==","Attempts":2,"MaxAttempts":5,' \
         b'"NotBefore":"2024-01-02T03:04:05.123456789Z"}'
    t2 = Task.decode(go)
    assert t2.payload == b'{"b":2}' and t2.attempts == 2 and t2.not_before.microsecond == 123456


def test_next_retry_schedule():
    now = dt.datetime(2024, 1, 1, tzinfo=dt.timezone.utc)
    t = Task(type="parse")
    delays = []
    while True:
        n = next_retry(t, now)
        if n is None:
            break
        delays.append((n.not_before - now).total_seconds())
    assert delays == [2, 4, 8, 16] and t.attempts == 5 and t.max_attempts == 5


class FlakyQueue:
    def __init__(self, fails):
        self.fails, self.calls = fails, 0

    async def enqueue(self, task):
        self.calls += 1
        if self.calls <= self.fails:
            raise RuntimeError("enqueue failed")


def test_enqueue_with_retry(monkeypatch):
    sleeps = []

    async def fake_sleep(s):
        sleeps.append(s)
    monkeypatch.setattr(asyncio, "sleep", fake_sleep)
    q = FlakyQueue(2)
    asyncio.run(enqueue_with_retry(q, Task(type="parse"), 3, 0.2))
    assert q.calls == 3 and sleeps == pytest.approx([0.2, 0.4])
    q = FlakyQueue(5)
    with pytest.raises(RuntimeError):
        asyncio.run(enqueue_with_retry(q, Task(type="parse"), 3, 0.2))
    assert q.calls == 3


def test_inproc_queue_groups_and_buffering():
    async def go():
        bus = InProcBus()
        q = InProcQueue(bus, discard())
        # published before any worker subscribed: buffered (not lost like core NATS)
        for i in range(3):
            await q.enqueue(Task(type="parse", payload=str(i).encode()))
        got = {"a": [], "b": []}
        stop = asyncio.Event()

        def h(name):
            async def handler(t):
                got[name].append(int(t.payload))
            return handler
        w1 = asyncio.ensure_future(q.worker("parse", h("a"), stop))
        w2 = asyncio.ensure_future(q.worker("parse", h("b"), stop))
        await asyncio.sleep(0.05)
        for i in range(3, 9):
            await q.enqueue(Task(type="parse", payload=str(i).encode()))
        await asyncio.sleep(0.1)
        stop.set()
        await asyncio.gather(w1, w2)
        allv = sorted(got["a"] + got["b"])
        assert allv == list(range(9))  # each task delivered exactly once across the group
        assert got["a"] and got["b"]  # load balanced
    asyncio.run(go())


def test_inproc_retry_then_permanent_failure(monkeypatch):
    monkeypatch.setattr(inproc_mod, "next_retry", lambda t, now=None: _fast_retry(t))
    failed = []

    async def go():
        q = InProcQueue(InProcBus(), discard())
        stop = asyncio.Event()
        calls = []

        async def handler(t):
            calls.append(t.attempts)
            raise RuntimeError("nope")

        async def on_fail(t, err):
            failed.append((t.attempts, str(err)))
            stop.set()
        w = asyncio.ensure_future(q.worker("analyze", handler, stop, on_permanent_failure=on_fail))
        await q.enqueue(Task(type="analyze"))
        await asyncio.wait_for(w, 5)
        assert calls == [0, 1, 2, 3, 4]
    asyncio.run(go())
    assert failed and failed[0][0] == 5


def _fast_retry(t):
    t.attempts += 1
    if t.max_attempts == 0:
        t.max_attempts = 5
    if t.attempts < t.max_attempts:
        t.not_before = dt.datetime.now(dt.timezone.utc) + dt.timedelta(milliseconds=5)
        return t
    return None


def test_multipart_roundtrip():
    body, ct = multipart.build({"x": "1"}, {"file": ("a.txt", b"hello\r\nworld", "text/plain")})
    p = multipart.form_file(body, ct)
    assert p.filename == "a.txt" and p.data == b"hello\r\nworld" and p.content_type == "text/plain" and p.size == 12
    body, ct = multipart.build({}, {"file": ("doc.pdf", b"%PDF", None)})
    assert multipart.form_file(body, ct).content_type == ""
    with pytest.raises(multipart.MultipartError):
        multipart.form_file(body, "application/json")
    body, ct = multipart.build({"other": "x"}, {})
    with pytest.raises(multipart.MultipartError):
        multipart.form_file(body, ct)


def test_pdf_extraction():
    pdf = make_pdf(["First page line one\nline two", "Second (page)"])
    assert extract_text(pdf) == "First page line one\nline two\nSecond (page)\n"
    assert extract_text(make_pdf(["plain"], compress=False)) == "plain\n"
    with pytest.raises(Exception):
        extract_text(b"hello, not a pdf")
