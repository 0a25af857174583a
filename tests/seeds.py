"""Deterministic per-case seeds: zlib.crc32 of the case text (Python's hash() of a str is salted per process, so
tables drawn from it could not be replayed after a red run)."""
import zlib


def seed_of(text: str) -> int:
    return zlib.crc32(text.encode("utf-8"))
