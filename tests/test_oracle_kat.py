"""Pins the CPU oracle against the reference's own known-answer tests (restated in kat_cases)."""
import pytest

from tests import kat_cases


@pytest.mark.parametrize("case", kat_cases.ALL, ids=lambda f: f.__name__)
def test_oracle_kat(oracle_lib, case):
    case(oracle_lib)
