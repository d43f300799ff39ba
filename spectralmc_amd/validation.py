"""Pydantic construction wrapped in a Result (reference ``src/spectralmc/validation.py:17``)."""

from __future__ import annotations

from typing import TypeVar

from pydantic import BaseModel, ValidationError

from .result import Failure, Result, Success

TModel = TypeVar("TModel", bound=BaseModel)


def validate_model(model_cls: type[TModel], **data: object) -> Result[TModel, ValidationError]:
    try:
        return Success(model_cls(**data))
    except ValidationError as exc:
        return Failure(exc)


__all__ = ["validate_model"]
