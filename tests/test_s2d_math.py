"""Space-to-depth stem derivation (CPU, no GPU): the ResNet 7x7 s2 p3 conv over a 4-channel image
equals a 4x4 s1 conv over its space-to-depth-by-2 image with top/left padding 2 and bottom/right
padding 1, using the re-laid-out weight of csrc/kernels/conv.hip stem_w_s2d_kernel:

    x2[b][(dh*2 + dw)*4 + c][i][j] = x[b][c][2i + dh][2j + dw]
    w2[n][r][s][(dh*2 + dw)*4 + c] = w[n][c][2r + dh - 1][2s + dw - 1]   (0 outside the 7x7)

and the weight gradient maps back by the inverse index permutation (stem_wgrad_s2d_kernel)."""
import torch
import torch.nn.functional as F


def s2d(x4):
    B, C, H, W = x4.shape
    return x4.view(B, C, H // 2, 2, W // 2, 2).permute(0, 3, 5, 1, 2, 4).reshape(B, 4 * C, H // 2, W // 2)


def w_s2d(w4):
    N = w4.shape[0]
    w2 = torch.zeros(N, 4, 4, 16, dtype=w4.dtype)          # [n][r][s][(dh*2+dw)*4 + c]
    for r in range(4):
        for s in range(4):
            for dh in range(2):
                for dw in range(2):
                    kh, kw = 2 * r + dh - 1, 2 * s + dw - 1
                    if 0 <= kh < 7 and 0 <= kw < 7:
                        w2[:, r, s, (dh * 2 + dw) * 4:(dh * 2 + dw) * 4 + 4] = w4[:, :, kh, kw]
    return w2


def grad_from_s2d(g2):
    """[N][4][4][16] -> [N][4][7][7] (kernel layout [N][7][7][4] transposed to torch's)"""
    N = g2.shape[0]
    g = torch.zeros(N, 4, 7, 7, dtype=g2.dtype)
    for kh in range(7):
        for kw in range(7):
            r, dh, s, dw = (kh + 1) // 2, (kh + 1) % 2, (kw + 1) // 2, (kw + 1) % 2
            g[:, :, kh, kw] = g2[:, r, s, (dh * 2 + dw) * 4:(dh * 2 + dw) * 4 + 4]
    return g


def test_stem_s2d_forward_equivalence():
    torch.manual_seed(0)
    for H in (32, 46, 64):
        x = torch.randn(2, 3, H, H, dtype=torch.float64)
        w = torch.randn(8, 3, 7, 7, dtype=torch.float64)
        ref = F.conv2d(x, w, stride=2, padding=3)
        x4 = torch.cat([x, torch.zeros(2, 1, H, H, dtype=x.dtype)], 1)
        w4 = torch.cat([w, torch.zeros(8, 1, 7, 7, dtype=w.dtype)], 1)
        w2 = w_s2d(w4).permute(0, 3, 1, 2)                   # [n][16][r][s]
        y = F.conv2d(F.pad(s2d(x4), (2, 1, 2, 1)), w2)
        assert y.shape == ref.shape
        assert torch.allclose(y, ref, atol=1e-10)


def test_stem_s2d_weight_gradient_equivalence():
    torch.manual_seed(1)
    H = 30
    x = torch.randn(2, 3, H, H, dtype=torch.float64)
    dy = torch.randn(2, 8, H // 2, H // 2, dtype=torch.float64)
    w = torch.zeros(8, 3, 7, 7, dtype=torch.float64, requires_grad=True)
    (gref,) = torch.autograd.grad(F.conv2d(x, w, stride=2, padding=3), w, dy)
    x4 = torch.cat([x, torch.zeros(2, 1, H, H, dtype=x.dtype)], 1)
    w2 = torch.zeros(8, 16, 4, 4, dtype=torch.float64, requires_grad=True)
    (g2,) = torch.autograd.grad(F.conv2d(F.pad(s2d(x4), (2, 1, 2, 1)), w2), w2, dy)
    g = grad_from_s2d(g2.permute(0, 2, 3, 1))               # [n][r][s][16] -> [n][4][7][7]
    assert torch.allclose(g[:, :3], gref, atol=1e-10)
    assert g[:, 3].abs().max().item() == 0.0
