"""Success / Failure result type used across the public API.

Mirrors the reference's ``Result`` ADT (reference ``src/spectralmc/result.py``): frozen
value carriers that support structural pattern matching (``case Success(v)``) plus the
combinators the reference API exposes (``unwrap``, ``map``, ``collect_results``,
``fold_results`` ...).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Generic, NoReturn, TypeVar, Union

T = TypeVar("T")
U = TypeVar("U")
E = TypeVar("E")
F = TypeVar("F")


@dataclass(frozen=True)
class Success(Generic[T]):
    value: T

    def is_success(self) -> bool:
        return True

    def is_failure(self) -> bool:
        return False

    def unwrap(self) -> T:
        return self.value

    def unwrap_or(self, default: T) -> T:
        return self.value

    def unwrap_or_else(self, f: Callable[[object], T]) -> T:
        return self.value

    def map(self, f: Callable[[T], U]) -> "Result[U, object]":
        return Success(f(self.value))

    def map_error(self, f: Callable[[object], F]) -> "Result[T, F]":
        return self

    def flat_map(self, f: Callable[[T], "Result[U, E]"]) -> "Result[U, E]":
        return f(self.value)

    and_then = flat_map


@dataclass(frozen=True)
class Failure(Generic[E]):
    error: E

    def is_success(self) -> bool:
        return False

    def is_failure(self) -> bool:
        return True

    def unwrap(self) -> NoReturn:
        raise RuntimeError(f"called unwrap() on Failure: {self.error!r}")

    def unwrap_or(self, default: T) -> T:
        return default

    def unwrap_or_else(self, f: Callable[[E], T]) -> T:
        return f(self.error)

    def map(self, f: Callable[[object], U]) -> "Result[U, E]":
        return self

    def map_error(self, f: Callable[[E], F]) -> "Result[object, F]":
        return Failure(f(self.error))

    def flat_map(self, f: Callable[[object], "Result[U, E]"]) -> "Result[U, E]":
        return self

    and_then = flat_map


Result = Union[Success[T], Failure[E]]


def expect(result: "Result[T, E]") -> T:
    if isinstance(result, Success):
        return result.value
    raise RuntimeError(f"expected Success, got Failure({result.error!r})")


def collect_results(results: "list[Result[T, E]]") -> "Result[list[T], E]":
    """First Failure wins; otherwise the list of values."""
    values: list[T] = []
    for res in results:
        if isinstance(res, Failure):
            return res
        values.append(res.value)
    return Success(values)


def partition_results(results: "list[Result[T, E]]") -> tuple[list[T], list[E]]:
    ok = [r.value for r in results if isinstance(r, Success)]
    bad = [r.error for r in results if isinstance(r, Failure)]
    return ok, bad


def fold_results(items: list[T], f: Callable[[U, T], "Result[U, E]"], initial: U) -> "Result[U, E]":
    """Left fold that stops at the first Failure."""
    acc: U = initial
    for item in items:
        step = f(acc, item)
        if isinstance(step, Failure):
            return step
        acc = step.value
    return Success(acc)


__all__ = ["Success", "Failure", "Result", "expect", "collect_results", "partition_results", "fold_results"]
