"""Static checks of the compiled conv kernels (no GPU): the K loops of the hot fp32 (x3) kernels
must not touch scratch memory.  A cursor change once pushed the x3 3x3 forward's main loop into
scratch (6-7 scratch stores per K step) and cost ~35 % of those kernels in the step
(docs/DESIGN.md §4d); this catches that class of regression at build time.

Reads the object files of the in-tree build (mx_rcnn_amd/csrc/_build) with the ROCm LLVM tools;
skipped when either is missing."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
BUILD = os.path.join(ROOT, 'mx_rcnn_amd', 'csrc', '_build')

# (object, mangled-name substring): the x3 64x64 forward tiles (ring depth 3 and 2) and the grouped
# x3 data + weight gradient launch
KERNELS = [
    ('conv_igemm.hip.o', 'conv_igemm_buf_kernelILi64ELi64ELi3ELb0ELb1ELb0ELb1E'),
    ('conv_igemm.hip.o', 'conv_igemm_buf_kernelILi64ELi64ELi2ELb0ELb1ELb0ELb1E'),
    ('conv_igemm.hip.o', 'conv_dgrad_wgrad_kernelILi2ELb1ELb1ELi1ELb1E'),
]


def _tools_ok():
    from tools import isa_loop
    return all(os.path.exists(os.path.join(isa_loop.LLVM, t))
               for t in ('llvm-objcopy', 'clang-offload-bundler', 'llvm-objdump', 'llvm-readelf'))


_ASM = {}


def _asm(obj, tmp):
    from tools import isa_loop
    if obj not in _ASM:
        _ASM[obj] = isa_loop.disassemble(os.path.join(BUILD, obj), tmp)[0]
    return _ASM[obj]


@pytest.mark.parametrize('obj,name', KERNELS)
def test_hot_conv_loops_do_not_spill(obj, name, tmp_path):
    from tools import isa_loop
    if not os.path.exists(os.path.join(BUILD, obj)) or not _tools_ok():
        pytest.skip('no in-tree build objects or ROCm LLVM tools')
    asm = _asm(obj, str(tmp_path))
    if name not in asm:
        pytest.skip('kernel %s not in this build' % name)
    _, n, loops = isa_loop.loops(asm, name)
    assert n > 0 and loops, 'no MFMA loop found in %s' % name
    for j, i, ln, c in loops:
        assert c['scratch_store'] == 0 and c['scratch_load'] == 0, (name, j, i, dict(c))
