"""Versioned checkpoint store on a local filesystem (offline stand-in for the reference's
S3 store, storage/store.py:200-907, with the same object layout and commit semantics).

Layout under ``root`` (the reference's bucket keys):
    chain.json                               head record (ModelVersion fields)
    versions/<v##########_semver_hash8>/     checkpoint.pb, metadata.json, content_hash.txt
    audit/log.jsonl                          append-only commit log

Commit = write the version's artifacts, then compare-and-swap the head under an exclusive
file lock: if the head moved since the commit read it, the artifacts are rolled back and
``ConflictError`` is raised (store.py:596-790).  Blocking file IO runs in worker threads.
"""

from __future__ import annotations

import asyncio
import fcntl
import hashlib
import json
import os
import shutil
import tempfile
from pathlib import Path

from ..result import Failure, Result, Success
from .chain import ModelVersion, create_genesis_version, next_version
from .errors import (
    ChainCorruptionError,
    ChecksumError,
    CommitError,
    ConflictError,
    HeadNotFoundError,
    VersionNotFoundError,
)


def sha256_hex(data: bytes) -> str:
    return hashlib.sha256(data).hexdigest()


def _atomic_write(path: Path, data: bytes) -> None:
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = path.with_name(path.name + ".tmp")
    with open(tmp, "wb") as f:
        f.write(data)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


class AsyncBlockchainModelStore:
    """``async with AsyncBlockchainModelStore(root) as store: await store.commit(...)``."""

    def __init__(self, root: str | os.PathLike[str] | None = None, bucket_name: str = "opt-models") -> None:
        self.bucket_name = bucket_name
        self._owns_root = root is None
        self.root = Path(root) if root is not None else Path(tempfile.mkdtemp(prefix="smc-store-"))
        self.root.mkdir(parents=True, exist_ok=True)

    async def __aenter__(self) -> "AsyncBlockchainModelStore":
        return self

    async def __aexit__(self, *exc: object) -> None:
        return None

    def cleanup(self) -> None:
        """Remove a store created in a temporary directory."""
        if self._owns_root:
            shutil.rmtree(self.root, ignore_errors=True)

    # ---------------------------------------------------------------- blocking helpers
    @property
    def _chain(self) -> Path:
        return self.root / "chain.json"

    def _read_head(self) -> ModelVersion | None:
        if not self._chain.exists():
            return None
        return ModelVersion.from_json(json.loads(self._chain.read_text()))

    def _commit_sync(self, data: bytes, content_hash: str, message: str) -> ModelVersion:
        actual = sha256_hex(data)
        if actual != content_hash:
            raise ChecksumError(content_hash, actual)
        head = self._read_head()
        version = (create_genesis_version(content_hash, message or "Genesis version") if head is None
                   else next_version(head, content_hash, message))
        vdir = self.root / "versions" / version.directory_name
        try:
            _atomic_write(vdir / "checkpoint.pb", data)
            _atomic_write(vdir / "metadata.json", json.dumps(version.to_json(), indent=2).encode())
            _atomic_write(vdir / "content_hash.txt", content_hash.encode())
        except OSError as exc:
            shutil.rmtree(vdir, ignore_errors=True)
            raise CommitError(f"Failed to write artifacts: {exc}") from exc
        lock_path = self.root / ".chain.lock"
        with open(lock_path, "a+") as lock:
            fcntl.flock(lock, fcntl.LOCK_EX)
            try:
                now = self._read_head()
                moved = (now is None) != (head is None) or (now is not None and head is not None
                                                            and now.content_hash != head.content_hash)
                if moved:
                    shutil.rmtree(vdir, ignore_errors=True)
                    raise ConflictError("Concurrent commit detected: head moved during commit")
                _atomic_write(self._chain, json.dumps(version.to_json(), indent=2).encode())
            finally:
                fcntl.flock(lock, fcntl.LOCK_UN)
        log = self.root / "audit" / "log.jsonl"
        log.parent.mkdir(parents=True, exist_ok=True)
        with open(log, "a") as f:
            f.write(json.dumps({"version_id": version.version_id, **version.to_json()}) + "\n")
        return version

    def _version_dir(self, version_id: str) -> Path:
        vroot = self.root / "versions"
        if vroot.exists():
            for d in sorted(vroot.iterdir()):
                if d.name.startswith(version_id + "_"):
                    return d
        raise VersionNotFoundError(version_id)

    def _get_version_sync(self, version_id: str) -> ModelVersion:
        return ModelVersion.from_json(json.loads((self._version_dir(version_id) / "metadata.json").read_text()))

    def _load_sync(self, version: ModelVersion) -> bytes:
        path = self.root / "versions" / version.directory_name / "checkpoint.pb"
        if not path.exists():
            raise VersionNotFoundError(version.version_id)
        data = path.read_bytes()
        actual = sha256_hex(data)
        if actual != version.content_hash:
            raise ChecksumError(version.content_hash, actual)
        return data

    def _list_sync(self) -> list[ModelVersion]:
        vroot = self.root / "versions"
        if not vroot.exists():
            return []
        out = [ModelVersion.from_json(json.loads((d / "metadata.json").read_text()))
               for d in vroot.iterdir() if (d / "metadata.json").exists()]
        return sorted(out, key=lambda v: v.counter)

    # ---------------------------------------------------------------- async API
    async def get_head(self) -> Result[ModelVersion, HeadNotFoundError]:
        head = await asyncio.to_thread(self._read_head)
        return Success(head) if head is not None else Failure(HeadNotFoundError("no commits yet"))

    async def commit(self, checkpoint_data: bytes, content_hash: str, message: str = "") -> ModelVersion:
        return await asyncio.to_thread(self._commit_sync, checkpoint_data, content_hash, message)

    async def get_version(self, version_id: str) -> ModelVersion:
        return await asyncio.to_thread(self._get_version_sync, version_id)

    async def load_checkpoint(self, version: ModelVersion) -> bytes:
        return await asyncio.to_thread(self._load_sync, version)

    async def list_versions(self) -> list[ModelVersion]:
        return await asyncio.to_thread(self._list_sync)

    async def verify_chain(self) -> list[ModelVersion]:
        """Check counters are 0..n-1, parents link by content hash and the head is the last."""
        versions = await self.list_versions()
        for i, v in enumerate(versions):
            if v.counter != i:
                raise ChainCorruptionError(f"counter gap at {v.version_id}")
            want_parent = "" if i == 0 else versions[i - 1].content_hash
            if v.parent_hash != want_parent:
                raise ChainCorruptionError(f"broken parent link at {v.version_id}")
        head = await asyncio.to_thread(self._read_head)
        if versions and (head is None or head.compute_hash() != versions[-1].compute_hash()):
            raise ChainCorruptionError("head does not point at the last version")
        return versions


__all__ = ["AsyncBlockchainModelStore", "sha256_hex"]
