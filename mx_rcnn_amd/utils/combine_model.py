"""Union of two checkpoints, first wins on duplicates (reference `utils/combine_model.py:5-22`);
used by alternate training to merge RPN2 + RCNN into the final model."""
from .load_model import load_checkpoint, save_checkpoint


def combine_model(prefix1, epoch1, prefix2, epoch2, prefix_out, epoch_out):
    args1, auxs1 = load_checkpoint(prefix1, epoch1)
    args2, auxs2 = load_checkpoint(prefix2, epoch2)
    args = dict(args2)
    args.update(args1)
    auxs = dict(auxs2)
    auxs.update(auxs1)
    save_checkpoint(prefix_out, epoch_out, args, auxs)
    return args, auxs
