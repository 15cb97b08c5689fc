"""Host-side argument validation of the HIP op wrappers (no GPU needed: the checks run
before any kernel launch)."""
import pytest
import torch

import pgdist  # noqa: F401
from pgdist.ops import kernels as K


@pytest.mark.parametrize("px", [-1, 3, 8])
def test_stem_px_rejected(px):
    t = torch.zeros(1)
    with pytest.raises(ValueError, match="px"):
        K.stem_fwd(t, t, t, t, 1, 32, 32, px=px)


def test_operands_of_2gib_or_more_rejected():
    """32-bit buffer offsets with the 0x80000000 mask offset: operands must stay below 2 GiB."""
    big = torch.zeros(1, dtype=torch.uint8).expand(1 << 31)        # 2 GiB, no storage behind it
    with pytest.raises(ValueError, match="2 GiB"):
        K._p(big)
    ok = torch.zeros(1, dtype=torch.uint8).expand((1 << 31) - 1)
    assert K._p(ok) == ok.data_ptr()
