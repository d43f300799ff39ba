"""Snapshot <-> checkpoint bytes <-> store (reference storage/checkpoint.py:45-188)."""

from __future__ import annotations

from ..models.torch import build_adam_optimizer_state
from ..result import Failure, Result, Success
from .chain import ModelVersion
from .errors import SerializationFailure
from .store import AsyncBlockchainModelStore, sha256_hex
from .wire import checkpoint_from_proto, checkpoint_to_proto, messages


def create_checkpoint_from_snapshot(snapshot) -> tuple[bytes, str]:
    """Serialise a ``GbmCVNNPricerConfig`` snapshot to ModelCheckpointProto bytes + SHA-256."""
    opt = snapshot.optimizer_state
    if opt is None:
        empty = build_adam_optimizer_state(param_states={}, param_groups=[])
        if isinstance(empty, Failure):
            raise RuntimeError(f"Failed to create empty optimizer state: {empty.error}")
        opt = empty.value
    msg = checkpoint_to_proto(snapshot.cvnn.state_dict(), opt, snapshot.torch_cpu_rng_state or b"",
                              list(snapshot.torch_cuda_rng_states or []), snapshot.global_step)
    if isinstance(msg, Failure):
        raise RuntimeError(f"Failed to serialize checkpoint: {msg.error}")
    data = msg.value.SerializeToString()
    return data, sha256_hex(data)


async def commit_snapshot(store: AsyncBlockchainModelStore, snapshot, message: str = "") -> ModelVersion:
    data, content_hash = create_checkpoint_from_snapshot(snapshot)
    return await store.commit(checkpoint_data=data, content_hash=content_hash, message=message)


async def load_snapshot_from_checkpoint(store: AsyncBlockchainModelStore, version: ModelVersion, cvnn_template,
                                        cfg) -> Result[object, SerializationFailure]:
    """Load ``version`` into ``cvnn_template``; the simulation config, domain bounds and Sobol
    position come from ``cfg``, everything else from the checkpoint."""
    from ..gbm_trainer import ComplexValuedModel, build_gbm_cvnn_pricer_config

    data = await store.load_checkpoint(version)
    msg = messages()["ModelCheckpointProto"]()
    msg.ParseFromString(data)
    parts = checkpoint_from_proto(msg)
    if isinstance(parts, Failure):
        return parts
    state_dict, opt, cpu_rng, cuda_rngs, global_step = parts.value
    cvnn_template.load_state_dict(state_dict)
    if not isinstance(cvnn_template, ComplexValuedModel):
        raise TypeError(f"cvnn_template must implement ComplexValuedModel, got {type(cvnn_template).__name__}")
    built = build_gbm_cvnn_pricer_config(cfg=cfg.cfg, domain_bounds=cfg.domain_bounds, cvnn=cvnn_template,
                                         optimizer_state=opt if opt.param_states else None, global_step=global_step,
                                         sobol_skip=cfg.sobol_skip, torch_cpu_rng_state=cpu_rng or None,
                                         torch_cuda_rng_states=cuda_rngs or None)
    if isinstance(built, Failure):
        return Failure(SerializationFailure(message=f"invalid snapshot: {built.error}"))
    return Success(built.value)


__all__ = ["create_checkpoint_from_snapshot", "commit_snapshot", "load_snapshot_from_checkpoint"]
