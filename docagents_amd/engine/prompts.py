"""Prompts, verbatim from the reference (internal/llm/openai.go:47 and :71-78, :82)."""
from ..text.preprocess import go_fields

SUMMARIZE_SYSTEM = ("You are a concise assistant. First provide a brief summary paragraph, then list the key "
                    "points as bullet points (using - or *).")

ANSWER_SYSTEM = """You are a precise document Q&A assistant. Follow these rules strictly:

1. Answer ONLY using information from the provided context
2. If the answer is not in the context, respond with "I don't have enough information to answer this question"
3. Cite specific parts of the context when answering (e.g., "According to the documentation...")
4. Be concise but complete - include all relevant details from the context
5. If the context contains conflicting information, mention both perspectives
6. Never make assumptions or add information not present in the context"""


def answer_user(context: str, question: str) -> str:
    return f"Context:\n{context}\n\nQuestion: {question}"


def build_context(chunk_texts: list[str]) -> str:
    """cmd/query/main.go:150-157: chunk texts each followed by a newline."""
    return "".join(t + "\n" for t in chunk_texts)


def concatenate_chunks(chunk_texts: list[str]) -> str:
    """cmd/analysis/main.go:115-122."""
    return "".join(t + "\n" for t in chunk_texts)


def dedup_overlap(chunk_texts: list[str], max_overlap: int) -> list[str]:
    """Drop from every chunk the leading words it shares with the end of the previous chunk (the
    chunker's sliding-window overlap, 80 words by default). The reference summarizes the raw
    concatenation (cmd/analysis/main.go:115-122), i.e. ~25 % duplicated words at 400/80; SURVEY §5.7 /
    Appendix B #7-8: the summary input carries each word span once, in ``ord`` order. Chunks hold
    single-space-joined words (text/chunker.py), so the overlap is found by exact word match."""
    out: list[str] = []
    prev: list[str] = []
    for i, t in enumerate(chunk_texts):
        words = go_fields(t)
        k = 0
        if i > 0 and max_overlap > 0:
            for n in range(min(max_overlap, len(prev), len(words)), 0, -1):
                if words[:n] == prev[-n:]:
                    k = n
                    break
        rest = words[k:]
        if rest:
            out.append(" ".join(rest) if k else t)
        prev = words
    return out


def enrich_for_embedding(filename: str, text: str) -> str:
    """cmd/analysis/main.go:89-93."""
    return f"Document: {filename}\n\n{text}"
