"""Shared plumbing for the CLI entry points (train_end2end.py, train_alternate.py,
train_widerface*.py, test.py, tools/*): process-group bootstrap, roidb construction (VOC,
.lst, synthetic), model construction + pretrained loading + new-layer initialisation
(`train_end2end.py:56-78`), optimizer parameters (`train_end2end.py:98-105`), frozen prefixes.

Multi-GPU: ``--gpus 0,1,2,3`` names DEVICES, as the reference's device list does
(`train_end2end.py:168`): one process per listed device from the single command
(parallel/spawn.py: fresh child processes, torchrun's environment contract), ``--gpus 3`` one
process on device 3.  The ids index the devices the job can see: under an existing
HIP_VISIBLE_DEVICES mask, id i is the mask's i-th entry.  Under ``torchrun --nproc-per-node N``
the launcher's ranks are used as they are.  The device of each rank is its LOCAL_RANK.  Gradients
are summed across ranks like the reference's kvstore (rescale_grad 1.0).
"""
import logging
import os

import numpy as np
import torch

from ..config import config, override, parse_cfg_overrides, snapshot
from ..models import FasterRCNN
from ..parallel import dist as pdist
from ..utils.load_model import load_param
from .lr_scheduler import FactorScheduler, WarmupScheduler

FIXED_PREFIX = {'vgg': ['conv1', 'conv2'], 'resnet': ['conv0', 'stage1', 'stage2', 'bn_data', 'bn0']}


def setup_logging(rank=0):
    logging.basicConfig(level=logging.INFO if rank == 0 else logging.WARNING,
                        format='%(asctime)s %(levelname)s %(message)s')


def add_common_args(parser, eval_cli=False):
    """The flags every CLI shares.  ``eval_cli``: --dtype is the TEST graph's precision (fp32 = the
    reference's, as exact three-plane bf16 operands on the MFMA kernels; bf16; fp16)."""
    parser.add_argument('--network', default='vgg16', help='vgg16 | resnet18..resnet200')
    parser.add_argument('--synthetic', type=int, default=0, help='use N synthetic images instead of a dataset')
    parser.add_argument('--synthetic-shape', default='600x1000')
    parser.add_argument('--synthetic-kind', default='noise', choices=('noise', 'planted'),
                        help='noise: benchmark-shaped random images; planted: learnable class-specific objects '
                             '(train on one --seed, test on another)')
    parser.add_argument('--cfg', nargs='*', default=[], help='config overrides key=value (e.g. TRAIN.RPN_MIN_SIZE=10)')
    parser.add_argument('--max-steps', type=int, default=None, help='stop after this many steps (smoke runs)')
    parser.add_argument('--eager', action='store_true', help='disable hipGraph step capture')
    parser.add_argument('--ims-per-gpu', type=int, default=1)
    parser.add_argument('--seed', type=int, default=0)
    if eval_cli:
        parser.add_argument('--dtype', default='fp32', choices=('fp32', 'bf16', 'fp16'),
                            help='test-graph precision on the GPU (core/detector.py): fp32 = the reference '
                                 'precision (exact fp32 triples on the MFMA kernels), bf16 / fp16 operands with '
                                 'fp32 accumulation')
        return parser
    parser.add_argument('--dtype', default='fp32', choices=('fp32', 'bf16x3', 'bf16'),
                        help='training precision on the GPU (ops/precision.py): fp32 = the reference '
                             'precision (exact fp32 triples, six bf16 products), bf16x3 = 16-bit pairs, '
                             'bf16 = bf16 operands; fp32 accumulation, gradients and masters in all')
    return parser


def init_runtime(args):
    """Spawn the per-GPU ranks if ``--gpus`` names more than one device (the parent exits with
    the job's code and never touches the GPU), then bootstrap this rank."""
    from ..parallel.spawn import maybe_spawn, parse_gpus, select_devices
    import sys
    spec = getattr(args, 'gpus', None)
    if spec is None:
        spec = getattr(args, 'gpu_ids', None)
    if spec is not None:
        # --gpus names DEVICES as in the reference ('2,3' runs on GPUs 2 and 3, '3' on GPU 3)
        maybe_spawn(parse_gpus(spec), sys.argv[0], sys.argv[1:], visible=select_devices(spec))
    rank, world, local_rank, device = pdist.init_distributed()
    setup_logging(rank)
    if getattr(args, 'dtype', None):
        from ..ops import precision
        if args.dtype in precision.PLANES:  # a training precision (eval CLIs also take fp16)
            precision.set_default(args.dtype)
    if getattr(args, 'cfg', None):
        override(parse_cfg_overrides(args.cfg))
    torch.manual_seed(getattr(args, 'seed', 0) + rank)
    np.random.seed(getattr(args, 'seed', 0) + rank)
    return rank, world, device


def family(network):
    return 'resnet' if network.startswith('resnet') else 'vgg'


def build_model(network, num_classes, pretrained=None, load_epoch=0, resume=False, bn_mom=0.99, train_mode='e2e'):
    """Model with MXNet names; loads ``pretrained-%04d.params`` when it exists, drops the
    ImageNet classifier, re-initialises the new detection layers unless resuming."""
    model = FasterRCNN(network, num_classes, cfg=snapshot(), bn_mom=bn_mom, train_mode=train_mode)
    arg = aux = None
    if pretrained and pretrained.lower() != 'none':
        path = '%s-%04d.params' % (pretrained, load_epoch)
        if os.path.exists(path):
            arg, aux, _ = load_param(pretrained, load_epoch, convert=False)
            for k in ('fc8_weight', 'fc8_bias', 'fc1_weight', 'fc1_bias'):
                arg.pop(k, None)
            if not resume:
                for k in [k for k in arg if k.startswith('rpn_') or k.startswith('cls_score') or
                          k.startswith('bbox_pred')]:
                    arg.pop(k)  # keep the fresh N(0, 0.01) / N(0, 0.001) initialisation
            logging.info('loaded pretrained %s (%d args, %d aux)', path, len(arg), len(aux))
        else:
            logging.warning('pretrained %s not found: random initialisation', path)
    return model, arg, aux


def optimizer_params(lr, mom, wd, factor_step, resume, warmup=True):
    sched = FactorScheduler(factor_step, 0.1) if (resume or not warmup) else \
        WarmupScheduler(factor_step, 0.1, warmup_lr=0.1 * lr, warmup_step=200)
    return {'momentum': mom, 'wd': wd, 'learning_rate': lr, 'lr_scheduler': sched, 'clip_gradient': 1.0,
            'rescale_grad': 1.0}


def e2e_config():
    """Run-time mutation of train_end2end.py:25-32."""
    config.TRAIN.BG_THRESH_LO = 0.0
    config.TRAIN.HAS_RPN = True
    config.END2END = 1
    config.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True


def synthetic_roidb(args, num_classes, flip=False):
    from ..data.load_data import load_synthetic_roidb
    h, w = [int(v) for v in args.synthetic_shape.lower().split('x')]
    config.SCALES = (min(h, w),)
    config.MAX_SIZE = max(h, w)
    return load_synthetic_roidb(args.synthetic, h, w, num_classes, flip=flip, seed=args.seed,
                                kind=getattr(args, 'synthetic_kind', 'noise'))


def raw_images(device):
    """Training loaders ship uint8 images converted on the device (ops/image.py) when training on
    the GPU (MXR_RAW_IMAGES=0: the host float path of the reference)."""
    return torch.device(device).type == 'cuda' and os.environ.get('MXR_RAW_IMAGES', '1') != '0'


def batch_images(b):
    """The network input of a loader batch (converts a raw uint8 batch on the CPU)."""
    x = torch.as_tensor(b['data'])
    if x.dtype == torch.uint8:
        from ..ops.image import image_prep
        x = image_prep(x, torch.as_tensor(b['im_info']), b.get('pixel_means'), torch.float32, False)
    return x


def calibrate_if_random(model, loader, arg_params):
    """Random-init ResNets get data-dependent BN statistics from the first batch (a pretrained
    checkpoint carries real ones); without them 100+ pre-activation units blow up.  A random VGG16
    trunk gets a data-dependent (LSUV) filter scale for the same reason (FasterRCNN.calibrate_vgg)."""
    if arg_params:
        return False
    b = loader.get_batch()
    if not model.network.startswith('resnet'):
        model.calibrate_vgg(batch_images(b))
        logging.info('no pretrained weights: data-dependent (LSUV) init of the %s trunk', model.network)
        return True
    model.calibrate_bn(batch_images(b))
    logging.info('no pretrained weights: calibrated %s BN statistics on the first batch', model.network)
    return True
