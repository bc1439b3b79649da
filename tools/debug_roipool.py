"""Localise the fp32 RoIPool backward mismatch seen in tests (GPU)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mx_rcnn_amd.ops import need_ext  # noqa: E402


def ref_bwd(gout, arg, rois, B, C, H, W):
    gin = torch.zeros(B, C * H * W, dtype=torch.float64)
    R = gout.shape[0]
    go = gout.double().cpu().reshape(R, C, -1)
    a = arg.cpu().reshape(R, C, -1).long()
    for r in range(R):
        b = int(rois[r, 0])
        if b < 0:
            continue
        m = a[r] >= 0
        gin[b].index_add_(0, (torch.arange(C)[:, None] * H * W + a[r].clamp_min(0))[m], go[r][m])
    return gin.reshape(B, C, H, W)


def main():
    cuda = torch.device('cuda')
    ext = need_ext()
    g = torch.Generator().manual_seed(4)
    for dtype, C in [(torch.float32, 64), (torch.bfloat16, 64), (torch.float32, 1024), (torch.bfloat16, 1024)]:
        B, H, W, R = 2, 38, 50, 64
        feat = torch.randn(B, C, H, W, generator=g).to(cuda, dtype).contiguous(memory_format=torch.channels_last)
        xy = torch.rand(R, 2, generator=g) * torch.tensor([W * 16 * 0.8, H * 16 * 0.8])
        wh = torch.rand(R, 2, generator=g) * 200 + 1
        rois = torch.cat([torch.randint(0, B, (R, 1), generator=g).float(), xy, xy + wh], 1).to(cuda)
        out, arg = ext.roi_pool_fwd(feat, rois, 7, 7, 1 / 16)
        gout = torch.randn(out.shape, generator=g).to(cuda, dtype)
        gin = ext.roi_pool_bwd(gout, arg, rois, B, H, W)
        torch.cuda.synchronize()
        ref = ref_bwd(gout, arg, rois.cpu(), B, C, H, W)
        got = gin.double().cpu()
        bad = ~torch.isclose(got, ref, atol=3e-2, rtol=3e-2)
        print(dtype, C, 'gin strides', gin.stride(), 'arg strides', arg.stride(), 'gout strides', gout.stride(),
              'bad', int(bad.sum()), '/', bad.numel(), flush=True)
        if bad.any():
            idx = torch.nonzero(bad)[:5]
            for b_, c_, h_, w_ in idx.tolist():
                print('  at', (b_, c_, h_, w_), 'got', float(got[b_, c_, h_, w_]), 'ref', float(ref[b_, c_, h_, w_]))
            # is it a layout permutation?
            print('  sum got', float(got.sum()), 'sum ref', float(ref.sum()))


if __name__ == '__main__':
    main()
