"""Checkpoint wire format and the local model store.

Reference behaviour: storage/checkpoint.py:45-188, storage/store.py:596-907,
storage/chain.py:12-100, serialization/tensors.py:33-593; field table pinned by
tests/golden/proto_fields.json (extracted from the reference .proto files)."""

from __future__ import annotations

import json
import os

import pytest
import torch
from google.protobuf.descriptor import FieldDescriptor

from spectralmc_amd.result import Failure, Success
from spectralmc_amd.storage import (
    AsyncBlockchainModelStore,
    ChecksumError,
    ConflictError,
    HeadNotFoundError,
    VersionNotFoundError,
    commit_snapshot,
    create_checkpoint_from_snapshot,
    load_snapshot_from_checkpoint,
)
from spectralmc_amd.storage.store import sha256_hex
from spectralmc_amd.storage.wire import (
    adam_from_proto,
    adam_to_proto,
    messages,
    tensor_from_proto,
    tensor_to_proto,
)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "proto_fields.json")

_SCALAR = {FieldDescriptor.TYPE_DOUBLE: "double", FieldDescriptor.TYPE_INT64: "int64",
           FieldDescriptor.TYPE_UINT64: "uint64", FieldDescriptor.TYPE_INT32: "int32",
           FieldDescriptor.TYPE_UINT32: "uint32", FieldDescriptor.TYPE_BOOL: "bool",
           FieldDescriptor.TYPE_STRING: "string", FieldDescriptor.TYPE_BYTES: "bytes"}


def _type_name(f: FieldDescriptor) -> str:
    if f.message_type is not None and f.message_type.GetOptions().map_entry:
        k, v = f.message_type.fields_by_name["key"], f.message_type.fields_by_name["value"]
        return f"map<{_type_name(k)},{_type_name(v)}>"
    if f.type == FieldDescriptor.TYPE_MESSAGE:
        return f.message_type.name
    if f.type == FieldDescriptor.TYPE_ENUM:
        return f.enum_type.name
    return _SCALAR[f.type]


def test_descriptors_match_reference_field_table() -> None:
    with open(GOLDEN) as fh:
        table = json.load(fh)
    msgs = messages()
    assert set(table) == set(msgs)
    for name, fields in table.items():
        desc = msgs[name].DESCRIPTOR
        ours = sorted([f.name, f.number, _type_name(f), f.is_repeated and
                       not (f.message_type is not None and f.message_type.GetOptions().map_entry)]
                      for f in desc.fields)
        assert ours == sorted(fields), name
        assert desc.full_name == f"spectralmc.proto.{name}"


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.complex64, torch.complex128,
                                   torch.float16, torch.bfloat16])
def test_tensor_round_trip(dtype) -> None:
    t = (torch.randn(3, 5, dtype=torch.float64) * 3).to(dtype)
    msg = tensor_to_proto(t)
    assert isinstance(msg, Success)
    back = tensor_from_proto(type(msg.value).FromString(msg.value.SerializeToString()))
    assert isinstance(back, Success)
    assert back.value.dtype == dtype and back.value.shape == t.shape
    assert torch.equal(back.value.view(torch.uint8) if dtype == torch.bfloat16 else back.value,
                       t.view(torch.uint8) if dtype == torch.bfloat16 else t)


def test_tensor_encoding_layout() -> None:
    """Field 1 packed int64 shape, 2 dtype enum, 3 device enum, 4 raw little-endian bytes."""
    msg = tensor_to_proto(torch.tensor([1.0, 2.0], dtype=torch.float32)).value
    raw = msg.SerializeToString()
    data = torch.tensor([1.0, 2.0], dtype=torch.float32).numpy().tobytes()
    assert raw == bytes([0x0A, 0x01, 0x02, 0x10, 0x01, 0x18, 0x01, 0x22, 0x08]) + data


def test_adam_state_round_trip() -> None:
    p = [torch.nn.Parameter(torch.randn(4, 3)), torch.nn.Parameter(torch.randn(7))]
    opt = torch.optim.Adam(p, lr=3e-3, betas=(0.8, 0.95))
    for _ in range(3):
        opt.zero_grad()
        sum((x ** 2).sum() for x in p).backward()
        opt.step()
    from spectralmc_amd.models.torch import AdamOptimizerState

    state = AdamOptimizerState.from_torch(opt.state_dict()).value
    msg = adam_to_proto(state).value
    back = adam_from_proto(type(msg).FromString(msg.SerializeToString())).value
    assert back.param_groups[0].lr == 3e-3 and back.param_groups[0].betas == (0.8, 0.95)
    assert back.param_groups[0].params == [0, 1]
    for pid in (0, 1):
        assert back.param_states[pid].step == 3
        assert torch.equal(back.param_states[pid].exp_avg.to_torch().value, state.param_states[pid].exp_avg.to_torch().value)
    opt2 = torch.optim.Adam([torch.nn.Parameter(x.detach().clone()) for x in p], lr=1.0)
    opt2.load_state_dict(back.to_torch().value)  # loadable into a fresh optimizer


async def test_store_commit_chain_and_load(async_store: AsyncBlockchainModelStore) -> None:
    head = await async_store.get_head()
    assert isinstance(head, Failure) and isinstance(head.error, HeadNotFoundError)
    blobs = [b"alpha" * 10, b"beta" * 7, b"gamma"]
    versions = [await async_store.commit(b, sha256_hex(b), f"m{i}") for i, b in enumerate(blobs)]
    assert [v.counter for v in versions] == [0, 1, 2]
    assert [v.semantic_version for v in versions] == ["1.0.0", "1.0.1", "1.0.2"]
    assert versions[0].parent_hash == "" and versions[1].parent_hash == versions[0].content_hash
    assert versions[2].parent_hash == versions[1].content_hash
    assert versions[1].version_id == "v0000000001"
    assert versions[1].directory_name == f"v0000000001_1.0.1_{versions[1].content_hash[:8]}"
    head = await async_store.get_head()
    assert isinstance(head, Success) and head.value == versions[2]
    for v, b in zip(versions, blobs):
        assert await async_store.load_checkpoint(v) == b
    assert await async_store.get_version("v0000000001") == versions[1]
    assert await async_store.verify_chain() == versions
    with pytest.raises(VersionNotFoundError):
        await async_store.get_version("v0000000009")


async def test_store_rejects_corruption_and_bad_hash(async_store: AsyncBlockchainModelStore) -> None:
    with pytest.raises(ChecksumError):
        await async_store.commit(b"data", "0" * 64, "bad hash")
    v = await async_store.commit(b"data", sha256_hex(b"data"), "ok")
    path = async_store.root / "versions" / v.directory_name / "checkpoint.pb"
    path.write_bytes(b"tampered")
    with pytest.raises(ChecksumError):
        await async_store.load_checkpoint(v)


async def test_store_detects_concurrent_commit(async_store: AsyncBlockchainModelStore, monkeypatch) -> None:
    await async_store.commit(b"base", sha256_hex(b"base"), "base")
    real = async_store._read_head
    stale = real()
    calls = {"n": 0}

    def racing_read():
        calls["n"] += 1
        if calls["n"] == 1:  # the committer reads the head ...
            return stale
        return real()      # ... and by CAS time another writer has moved it

    await async_store.commit(b"other", sha256_hex(b"other"), "other writer")
    monkeypatch.setattr(async_store, "_read_head", racing_read)
    with pytest.raises(ConflictError):
        await async_store.commit(b"mine", sha256_hex(b"mine"), "loser")
    monkeypatch.undo()
    assert [v.commit_message for v in await async_store.verify_chain()] == ["base", "other writer"]


async def test_snapshot_commit_and_reload_cpu(async_store: AsyncBlockchainModelStore) -> None:
    """Snapshot-shaped object with a CPU CVNN: commit, reload into a different-seed template."""
    import types

    from spectralmc_amd.models.torch import AdamOptimizerState
    from tests.helpers import make_test_cvnn

    model = make_test_cvnn(n_inputs=6, n_outputs=16, seed=123, dtype=torch.float32, device="cpu")
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    x = torch.randn(4, 6)
    pr, pi = model(x, torch.zeros_like(x))
    (pr.square().mean() + pi.square().mean()).backward()
    opt.step()
    snap = types.SimpleNamespace(cvnn=model, optimizer_state=AdamOptimizerState.from_torch(opt.state_dict()).value,
                                 torch_cpu_rng_state=torch.get_rng_state().numpy().tobytes(),
                                 torch_cuda_rng_states=None, global_step=5)
    data, h = create_checkpoint_from_snapshot(snap)
    assert h == sha256_hex(data)
    v = await commit_snapshot(async_store, snap, "cpu snapshot")
    assert v.counter == 0 and v.commit_message == "cpu snapshot" and v.content_hash == h
    msg = messages()["ModelCheckpointProto"].FromString(await async_store.load_checkpoint(v))
    assert msg.global_step == 5 and set(msg.model_state_dict) == set(model.state_dict())
    template = make_test_cvnn(n_inputs=6, n_outputs=16, seed=999, dtype=torch.float32, device="cpu")
    from spectralmc_amd.storage.wire import checkpoint_from_proto

    sd, opt_state, cpu_rng, cuda_rngs, step = checkpoint_from_proto(msg).value
    template.load_state_dict(sd)
    for (k, a), b in zip(model.state_dict().items(), template.state_dict().values()):
        assert torch.equal(a, b), k
    assert cpu_rng == snap.torch_cpu_rng_state and cuda_rngs == [] and step == 5
    assert opt_state.param_states[0].step == 1
    assert load_snapshot_from_checkpoint is not None
