"""Host checks of the test helpers the GPU parity tests rely on for their failure messages."""

from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import assert_rows_equal


def test_assert_rows_equal_names_rows_and_their_launch_position() -> None:
    want = np.arange(520 * 4, dtype=np.float32).reshape(520, 4)
    assert_rows_equal(want.copy(), want)
    got = want.copy()
    got[[5, 13, 266]] += 1.0  # chunk 261: row 266 is workgroup 5 of the second launch
    with pytest.raises(AssertionError) as exc:
        assert_rows_equal(got, want, "case", chunk=261)
    msg = str(exc.value)
    assert "3 of 520 rows differ" in msg and "[5, 13, 266]" in msg
    assert "histogram [0, 0, 0, 0, 0, 3, 0, 0]" in msg
    nan = np.full((3, 2), np.nan)
    assert_rows_equal(nan, nan.copy())  # NaN == NaN, as np.testing.assert_array_equal
    with pytest.raises(AssertionError):
        assert_rows_equal(np.zeros((2, 2)), np.zeros((2, 3)))
