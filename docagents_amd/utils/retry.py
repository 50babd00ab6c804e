"""Exponential backoff (internal/retry/backoff.go:7-9): ``base * 2**attempt``, no jitter."""


def exponential_backoff(attempt: int, base: float) -> float:
    return base * (1 << attempt)
