"""CPU checks of the MXFP8 oracle (oracle/mx8_ref.py): the e4m3fn rounding against torch's
independent float8_e4m3fn cast, the OCP MX block rule, and the scale-layout round trip."""
import numpy as np
import torch

from oracle import mx8_ref


def _values(seed=0, n=200_000):
    rng = np.random.default_rng(seed)
    v = rng.standard_normal(n) * np.exp2(rng.integers(-14, 9, n))
    grid = mx8_ref.e4m3_decode(np.arange(256, dtype=np.uint8))
    grid = grid[np.isfinite(grid)]
    mids = (grid[:-1] + grid[1:]) / 2  # exact ties (RNE cases) of the sorted positive grid
    grid = np.sort(grid)
    mids = ((grid[:-1] + grid[1:]) / 2)
    return np.concatenate([v, grid, mids, -mids, [0.0, -0.0, 448.0, -448.0, 2.0 ** -9, 2.0 ** -10,
                                                   3 * 2.0 ** -11]]).astype(np.float32)


def test_e4m3_round_matches_torch():
    v = np.clip(_values(), -448, 448).astype(np.float32)
    ours = mx8_ref.e4m3_encode(mx8_ref.e4m3_round(v))
    ref = torch.from_numpy(v).to(torch.float8_e4m3fn).view(torch.uint8).numpy()
    nz = mx8_ref.e4m3_decode(ours) != 0  # torch may differ on the sign of zero only
    assert np.array_equal(ours[nz], ref[nz])
    assert np.all(mx8_ref.e4m3_decode(ref[~nz]) == 0)


def test_decode_encode_roundtrip():
    b = np.arange(256, dtype=np.uint8)
    b = b[(b & 0x7F) != 0x7F]  # NaNs
    assert np.array_equal(mx8_ref.e4m3_encode(mx8_ref.e4m3_decode(b)), b)


def test_block_rule():
    rng = np.random.default_rng(1)
    x = (rng.standard_normal((7, 256)) * np.exp2(rng.integers(-20, 20, (7, 1)))).astype(np.float32)
    x[3, 32:64] = 0.0  # an all-zero block
    q, sb = mx8_ref.quantize(x)
    assert sb[3, 1] == 0 and np.all(q[3, 32:64] & 0x7F == 0)
    deq = mx8_ref.dequantize(q, sb)
    blocks = np.abs(x).reshape(7, 8, 32).max(-1)
    # every block's largest element lands in [256, 512) * 2^(s - 127) before rounding
    lo = np.exp2(sb.astype(np.float64) - 127 + 8)
    nz = blocks > 0
    assert np.all(blocks[nz] >= lo[nz]) and np.all(blocks[nz] < 2 * lo[nz])
    # absolute error in a block <= half an ulp of its top binade (2^-4 amax), except for blocks whose
    # top element saturates from (448, 512) * X to 448 X (the OCP rule's clamp: <= 2^-3 amax)
    err = np.abs(deq - x).reshape(7, 8, 32).max(-1)
    sat = blocks >= 448 * lo / 256
    assert np.all(err[~sat] <= blocks[~sat] * 2.0 ** -4 + 1e-30)
    assert np.all(err[sat] <= blocks[sat] * 2.0 ** -3)


def test_scale_layout_roundtrip():
    rng = np.random.default_rng(2)
    sb = rng.integers(0, 255, (37, 24)).astype(np.uint8)
    s = mx8_ref.scales_to_dwords(sb, ld=40)
    assert s.shape == (6, 40)
    assert np.array_equal(mx8_ref.dwords_to_scales(s, 37), sb)
    # byte j of S[ks][r] is block 4 ks + j of row r
    assert (int(s[2, 5]) >> 8) & 0xFF == sb[5, 9]
