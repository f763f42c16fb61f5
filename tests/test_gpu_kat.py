"""The reference KATs (tests/kat_cases.py) against the HIP engine."""
import pytest

from tests import kat_cases

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", kat_cases.ALL, ids=lambda f: f.__name__)
def test_gpu_kat(gx_lib, case):
    case(gx_lib)
