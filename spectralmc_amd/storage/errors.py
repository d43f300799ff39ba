"""Storage errors (reference storage/errors.py:7-90: exception hierarchy; the wire layer's
failures are Result values as in errors/serialization.py)."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Literal


class StorageError(Exception):
    """Base class of store failures."""


class CommitError(StorageError):
    """A commit could not be completed."""


class NotFastForwardError(CommitError):
    """The new version's parent is not the current head."""


class ConflictError(CommitError):
    """A concurrent commit moved the head (compare-and-swap lost)."""


class ChecksumError(StorageError):
    """Stored checkpoint bytes do not hash to the version's content hash."""

    def __init__(self, expected: str, actual: str) -> None:
        super().__init__(f"checksum mismatch: expected {expected[:8]}, got {actual[:8]}")
        self.expected = expected
        self.actual = actual


class VersionNotFoundError(StorageError):
    def __init__(self, version_id: str) -> None:
        super().__init__(f"version not found: {version_id}")
        self.version_id = version_id


class ChainCorruptionError(StorageError):
    """Chain linkage (counter / parent hash) is broken."""


class HeadNotFoundError(StorageError):
    """The chain has no commits yet."""


@dataclass(frozen=True)
class SerializationFailure:
    message: str
    kind: Literal["SerializationFailure"] = "SerializationFailure"


__all__ = ["StorageError", "CommitError", "NotFastForwardError", "ConflictError", "ChecksumError",
           "VersionNotFoundError", "ChainCorruptionError", "HeadNotFoundError", "SerializationFailure"]
