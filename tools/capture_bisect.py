"""Capture progressively larger pieces of the training step into a hipGraph (one stage per
process, so a crash inside hipStreamEndCapture pinpoints the smallest failing piece)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mx_rcnn_amd.config import snapshot  # noqa: E402
from mx_rcnn_amd.models import FasterRCNN  # noqa: E402
from mx_rcnn_amd.core.trainer import Trainer  # noqa: E402


def main(stage):
    dev = torch.device('cuda')
    cfg = snapshot()
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    cfg.TRAIN.BG_THRESH_LO = 0.0
    # env knobs to replay other test configurations: MXR_BISECT_PRE/POST (proposal top-n),
    # MXR_BISECT_GTPAD=1 (a -1 padding gt row, as the tests' batches have)
    if os.environ.get('MXR_BISECT_PRE'):
        cfg.TRAIN.RPN_PRE_NMS_TOP_N = int(os.environ['MXR_BISECT_PRE'])
    if os.environ.get('MXR_BISECT_POST'):
        cfg.TRAIN.RPN_POST_NMS_TOP_N = int(os.environ['MXR_BISECT_POST'])
    torch.manual_seed(0)
    m = FasterRCNN('resnet50', 21, cfg=cfg)
    tr = Trainer(m, 'e2e', fixed_param_prefix=['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'], device=dev)
    H, W = 320, 480
    gt = [[20., 30, 200, 220, 3], [100, 50, 400, 300, 7]]
    if os.environ.get('MXR_BISECT_GTPAD') == '1':
        gt.append([-1., -1, -1, -1, -1])
    b = tr.prepare_batch({'data': torch.randn(1, 3, H, W) * 50, 'im_info': torch.tensor([[H, W, 1.0]]),
                          'gt_boxes': torch.tensor([gt]), 'n_gt': torch.tensor([2], dtype=torch.int32)})
    m.train()
    if stage in ('graphed', 'eager_then_graphed'):
        # the GraphedStep wrapper itself (tests/test_model.py::test_e2e_step_gpu_graph)
        from mx_rcnn_amd.core.trainer import GraphedStep
        if stage == 'eager_then_graphed':
            tr.step(b)
            torch.cuda.synchronize()
            print('[bisect] eager step done', flush=True)
        g = GraphedStep(tr, b, warmup=2)
        print('[bisect] captured', flush=True)
        for _ in range(3):
            g(b)
        torch.cuda.synchronize()
        print('[bisect] OK', stage, flush=True)
        return

    def fn():
        if stage == 'trunk_fwd':
            with torch.no_grad():
                m.trunk(b['data'])
        elif stage == 'trunk_fwdbwd':
            f = m.trunk(b['data'])
            f.float().sum().backward()
        elif stage == 'rpn_fwdbwd':
            out = m.train_rpn(b['data'], b['im_info'], b['gt_boxes'], b['n_gt'])
            out['loss'].backward()
        elif stage == 'e2e_fwd':
            with torch.no_grad():
                m.train_e2e(b['data'], b['im_info'], b['gt_boxes'], b['n_gt'])
        elif stage == 'e2e_fwdbwd':
            out = m.train_e2e(b['data'], b['im_info'], b['gt_boxes'], b['n_gt'])
            out['loss'].backward()
        elif stage == 'step':
            tr.step_body(b)
        else:
            raise ValueError(stage)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print('[bisect] OK', stage, flush=True)


if __name__ == '__main__':
    main(sys.argv[1])
