"""Version records of the model chain (reference storage/chain.py:12-100).

A version links to its parent by the parent's checkpoint content hash; its own record hash
covers every field, so rewriting history changes every later hash."""

from __future__ import annotations

import hashlib
from dataclasses import asdict, dataclass
from datetime import datetime, timezone


@dataclass(frozen=True)
class ModelVersion:
    counter: int
    semantic_version: str   # "MAJOR.MINOR.PATCH"
    parent_hash: str        # content hash of the parent version ("" for the genesis version)
    content_hash: str       # SHA-256 of checkpoint.pb
    commit_timestamp: str   # ISO-8601, UTC
    commit_message: str

    @property
    def version_id(self) -> str:
        return "v" + str(self.counter).zfill(10)

    @property
    def directory_name(self) -> str:
        return "_".join((self.version_id, self.semantic_version, self.content_hash[:8]))

    def compute_hash(self) -> str:
        fields = (self.counter, self.semantic_version, self.parent_hash, self.content_hash,
                  self.commit_timestamp, self.commit_message)
        return hashlib.sha256("|".join(str(f) for f in fields).encode()).hexdigest()

    def to_json(self) -> dict[str, object]:
        return asdict(self)

    @staticmethod
    def from_json(d: dict[str, object]) -> "ModelVersion":
        kinds = {"counter": int, "semantic_version": str, "parent_hash": str, "content_hash": str,
                 "commit_timestamp": str, "commit_message": str}
        for k, kind in kinds.items():
            if not isinstance(d.get(k), kind):
                raise TypeError(f"{k} must be {kind.__name__}, got {type(d.get(k)).__name__}")
        return ModelVersion(**{k: d[k] for k in kinds})  # type: ignore[arg-type]


def _utc_now() -> str:
    return datetime.now(timezone.utc).isoformat()


def bump_semantic_version(current: str, change_type: str = "patch") -> str:
    major, minor, patch = (int(x) for x in current.split("."))
    if change_type == "major":
        return f"{major + 1}.0.0"
    if change_type == "minor":
        return f"{major}.{minor + 1}.0"
    return f"{major}.{minor}.{patch + 1}"


def create_genesis_version(content_hash: str, message: str = "Genesis version") -> ModelVersion:
    return ModelVersion(counter=0, semantic_version="1.0.0", parent_hash="", content_hash=content_hash,
                        commit_timestamp=_utc_now(), commit_message=message)


def next_version(head: ModelVersion, content_hash: str, message: str) -> ModelVersion:
    return ModelVersion(counter=head.counter + 1, semantic_version=bump_semantic_version(head.semantic_version),
                        parent_hash=head.content_hash, content_hash=content_hash,
                        commit_timestamp=_utc_now(), commit_message=message)


__all__ = ["ModelVersion", "bump_semantic_version", "create_genesis_version", "next_version"]
