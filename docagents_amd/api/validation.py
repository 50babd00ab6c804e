"""Request decoding + validation with the reference's exact messages.

Go side: ``json.NewDecoder(r.Body).Decode(&req)`` into
``queryRequest{Question string validate:"required,min=3,max=500"; DocumentIDs []string
validate:"required,min=1,dive,uuid4"; TopK int validate:"omitempty,min=1,max=20"}``
(cmd/query/main.go:20-24,46-56) and ``formatFieldError`` (internal/httputil/httputil.go:128-144).
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass

# go-playground/validator uUID4Regex (lowercase hex only)
UUID4_RE = re.compile(r"^[0-9a-f]{8}-[0-9a-f]{4}-4[0-9a-f]{3}-[89ab][0-9a-f]{3}-[0-9a-f]{12}$")


class PayloadError(ValueError):
    pass


@dataclass
class QueryRequest:
    question: str = ""
    document_ids: list | None = None
    top_k: int = 0


def _go_key(d: dict, name: str):
    """encoding/json matches object keys to fields case-insensitively (exact match preferred)."""
    if name in d:
        return d[name]
    lname = name.lower()
    for k, v in d.items():
        if k.lower() == lname:
            return v
    return None


def decode_query_request(body: bytes) -> QueryRequest:
    try:
        text = body.decode("utf-8")
        obj, _ = json.JSONDecoder().raw_decode(text.lstrip())  # Decode reads ONE value
    except (UnicodeDecodeError, json.JSONDecodeError) as e:
        raise PayloadError(str(e)) from e
    req = QueryRequest()
    if obj is None:
        return req
    if not isinstance(obj, dict):
        raise PayloadError("json: cannot unmarshal into Go value of type main.queryRequest")
    q = _go_key(obj, "question")
    if q is not None:
        if not isinstance(q, str):
            raise PayloadError("json: cannot unmarshal into Go struct field queryRequest.question of type string")
        req.question = q
    ids = _go_key(obj, "document_ids")
    if ids is not None:
        if not isinstance(ids, list) or any(not isinstance(x, str) and x is not None for x in ids):
            raise PayloadError("json: cannot unmarshal into Go struct field queryRequest.document_ids")
        req.document_ids = ["" if x is None else x for x in ids]
    elif "document_ids" in obj:
        req.document_ids = None
    tk = _go_key(obj, "top_k")
    if tk is not None:
        if isinstance(tk, bool) or not isinstance(tk, (int, float)) or (isinstance(tk, float) and not tk.is_integer()):
            raise PayloadError("json: cannot unmarshal number into Go struct field queryRequest.top_k of type int")
        if isinstance(tk, float) and "." in json.dumps(tk):
            raise PayloadError("json: cannot unmarshal number into Go struct field queryRequest.top_k of type int")
        req.top_k = int(tk)
    return req


def validate_query_request(req: QueryRequest) -> list[str]:
    msgs = []
    # Question: required,min=3,max=500 (rune count)
    if req.question == "":
        msgs.append("Question is required")
    elif len(req.question) < 3:
        msgs.append("Question must be at least 3")
    elif len(req.question) > 500:
        msgs.append("Question must be at most 500")
    # DocumentIDs: required,min=1,dive,uuid4
    if req.document_ids is None:
        msgs.append("DocumentIDs is required")
    elif len(req.document_ids) < 1:
        msgs.append("DocumentIDs must be at least 1")
    else:
        for i, d in enumerate(req.document_ids):
            if not UUID4_RE.match(d):
                msgs.append(f"DocumentIDs[{i}] must be a valid UUID")
    # TopK: omitempty,min=1,max=20
    if req.top_k != 0:
        if req.top_k < 1:
            msgs.append("TopK must be at least 1")
        elif req.top_k > 20:
            msgs.append("TopK must be at most 20")
    return msgs
