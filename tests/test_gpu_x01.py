"""X01 packed payload kernels (csrc/kernels/x01.hip) == the torch reference packing, and the
pack → (W-rank int32 sum) → unpack round trip is exact on the device."""
import numpy as np
import pytest
import torch

from oni355 import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("V,KS,H,tail,W", [(1, 4, 0, 0, 1), (5733, 20, 300, 644, 8), (400_000, 20, 9000, 644, 2),
                                            (3000, 64, 0, 2052, 3), (170_000, 20, 2000, 644, 8)])
def test_x01_pack_unpack_kernels_match_reference(gpu, V, KS, H, tail, W):
    r = np.random.default_rng(V)
    O, O8 = 32767 // W, 127 // W
    perm = r.permutation(V)
    T = (V - H) * 3 // 4
    heavy = np.sort(perm[:H]).astype(np.int32)
    tiny = np.sort(perm[H:H + T]).astype(np.int32)
    light = np.sort(perm[H + T:]).astype(np.int32)
    hv, tv, lv = torch.from_numpy(heavy), torch.from_numpy(tiny), torch.from_numpy(light)
    n = ops.x01_packed_len(tv.numel(), lv.numel(), hv.numel(), KS, tail)
    dn = torch.from_numpy(r.integers(-O, O + 1, V * KS + tail).astype(np.int32))
    dn[: V * KS].view(V, KS)[tv.long()] = torch.from_numpy(r.integers(-O8, O8 + 1, (T, KS)).astype(np.int32))
    ref = torch.zeros(n, dtype=torch.int32)
    ops.x01_pack(dn, tv, lv, hv, KS, V * KS, tail, O8, O, ref)
    got = torch.zeros(n, dtype=torch.int32, device=gpu)
    ops.x01_pack(dn.to(gpu), tv.to(gpu), lv.to(gpu), hv.to(gpu), KS, V * KS, tail, O8, O, got)
    assert torch.equal(ref, got.cpu())
    # W identical contributions summed with int32 wrap-around, then unpacked on the device
    summed = ((ref.to(torch.int64) & 0xFFFFFFFF) * W % 2**32)
    summed = ((summed + 2**31) % 2**32 - 2**31).to(torch.int32)
    out = torch.zeros(V * KS + tail, dtype=torch.int32, device=gpu)
    ops.x01_unpack(summed.to(gpu), tv.to(gpu), lv.to(gpu), hv.to(gpu), KS, V * KS, tail, W * O8, W * O, out)
    assert torch.equal(out.cpu().to(torch.int64), dn.to(torch.int64) * W)
