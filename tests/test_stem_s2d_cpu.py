"""Space-to-depth stem algebra (csrc/kernels/stem.hip, ops/functional.py::
_StemS2DConvFn) in plain torch fp64: the 7x7/s2/pad-3 conv over 3 channels
equals a 4x4/s1 conv over the 2x2-blocked 16-channel image with pad (2 top/left,
1 bottom/right), using the kernel's channel order (dy*2+dx)*4 + c and tap map
i = 2r + dy - 1; and the weight-gradient fold inverts the weight map."""
import torch
import torch.nn.functional as F


def s2d_input(x):                       # x [N, H, W, 8] -> [N, H/2, W/2, 16]
    n, h, w, _ = x.shape
    q = x[..., :4].reshape(n, h // 2, 2, w // 2, 2, 4)          # n u dy v dx c
    return q.permute(0, 1, 3, 2, 4, 5).reshape(n, h // 2, w // 2, 16)


def s2d_weight(wt):                     # wt [K, C, 7, 7] -> [K, 4, 4, 16]
    K, C = wt.shape[:2]
    ws = torch.zeros(K, 4, 4, 16, dtype=wt.dtype)
    for r in range(4):
        for s in range(4):
            for dy in range(2):
                for dx in range(2):
                    i, j = 2 * r + dy - 1, 2 * s + dx - 1
                    if 0 <= i < 7 and 0 <= j < 7:
                        ws[:, r, s, (dy * 2 + dx) * 4:(dy * 2 + dx) * 4 + C] = wt[:, :, i, j]
    return ws


def fold(dws, C):                       # [K, 4, 4, 16] -> [K, C, 7, 7]
    K = dws.shape[0]
    dw = torch.zeros(K, C, 7, 7, dtype=dws.dtype)
    for i in range(7):
        for j in range(7):
            r, dy, s, dx = (i + 1) // 2, (i + 1) % 2, (j + 1) // 2, (j + 1) % 2
            dw[:, :, i, j] = dws[:, r, s, (dy * 2 + dx) * 4:(dy * 2 + dx) * 4 + C]
    return dw


def test_s2d_stem_forward_and_wgrad_fold():
    torch.manual_seed(0)
    N, H, K = 2, 16, 8
    x = torch.zeros(N, H, H, 8, dtype=torch.float64)
    x[..., :3] = torch.randn(N, H, H, 3, dtype=torch.float64)
    wt = torch.randn(K, 3, 7, 7, dtype=torch.float64)
    ref = F.conv2d(x[..., :3].permute(0, 3, 1, 2), wt, stride=2, padding=3)          # [N, K, 8, 8]
    xs = s2d_input(x).permute(0, 3, 1, 2)
    ws = s2d_weight(wt).permute(0, 3, 1, 2)
    y = F.conv2d(F.pad(xs, (2, 1, 2, 1)), ws)                                          # 4x4, s1
    torch.testing.assert_close(y, ref)
    # weight gradient: d(sum(y * g))/dws folded back == d/dwt of the 7x7 conv
    g = torch.randn_like(ref)
    dws = torch.nn.grad.conv2d_weight(F.pad(xs, (2, 1, 2, 1)), ws.shape, g)          # [K, 16, 4, 4]
    dwt = torch.nn.grad.conv2d_weight(x[..., :3].permute(0, 3, 1, 2), wt.shape, g, stride=2, padding=3)
    torch.testing.assert_close(fold(dws.permute(0, 2, 3, 1), 3), dwt)
