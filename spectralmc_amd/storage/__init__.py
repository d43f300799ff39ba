"""Versioned model checkpoints: the reference's wire format and chain
semantics over a local filesystem store (the reference's S3/MinIO backend, CLI, GC and
TensorBoard writer are out of scope)."""

from __future__ import annotations

from .chain import ModelVersion, bump_semantic_version, create_genesis_version
from .checkpoint import commit_snapshot, create_checkpoint_from_snapshot, load_snapshot_from_checkpoint
from .errors import (
    ChainCorruptionError,
    ChecksumError,
    CommitError,
    ConflictError,
    HeadNotFoundError,
    NotFastForwardError,
    StorageError,
    VersionNotFoundError,
)
from .store import AsyncBlockchainModelStore

__all__ = ["ModelVersion", "bump_semantic_version", "create_genesis_version", "commit_snapshot",
           "create_checkpoint_from_snapshot", "load_snapshot_from_checkpoint", "AsyncBlockchainModelStore",
           "StorageError", "CommitError", "NotFastForwardError", "ConflictError", "ChecksumError",
           "VersionNotFoundError", "ChainCorruptionError", "HeadNotFoundError"]
