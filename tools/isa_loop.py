"""Main-loop census of a compiled gfx950 kernel: the instruction mix of every loop body (a backward
branch) that holds MFMAs, plus the kernel's register / spill metadata -- the check that an edit to a
conv main loop did not make it spill (a scratch_store inside the K loop cost the x3 3x3 convs ~35 %
once: docs/DESIGN.md §4d).

    python tools/isa_loop.py mx_rcnn_amd/csrc/_build/conv_igemm.hip.o conv_igemm_buf_kernelILi64ELi64ELi3ELb0ELb1ELb0ELb1E

The object's offload bundle is extracted and disassembled with the ROCm LLVM tools
(/opt/rocm/lib/llvm/bin); the second argument is a substring of the mangled kernel name.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = os.path.join(os.environ.get('ROCM_PATH', '/opt/rocm'), 'lib', 'llvm', 'bin')


def disassemble(obj, tmp):
    fat, co = os.path.join(tmp, 'k.fatbin'), os.path.join(tmp, 'k.co')
    subprocess.run([os.path.join(LLVM, 'llvm-objcopy'), '--dump-section=.hip_fatbin=' + fat, obj, os.devnull],
                   check=True)
    subprocess.run([os.path.join(LLVM, 'clang-offload-bundler'), '--unbundle', '--type=o', '--input=' + fat,
                    '--targets=hipv4-amdgcn-amd-amdhsa--gfx950', '--output=' + co], check=True)
    asm = subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '-d', '--no-show-raw-insn', co], check=True,
                         stdout=subprocess.PIPE, text=True).stdout
    notes = subprocess.run([os.path.join(LLVM, 'llvm-readelf'), '--notes', co], check=True, stdout=subprocess.PIPE,
                           text=True).stdout
    return asm, notes


def kernel_meta(notes, name):
    """(vgpr_count, sgpr_count, vgpr_spill_count, sgpr_spill_count, private_segment_fixed_size)"""
    blocks = notes.split('  - .agpr_count:')
    for b in blocks:
        if re.search(r'\.name:\s+\S*%s' % re.escape(name), b):
            get = lambda k: (re.search(r'\.%s:\s+(\d+)' % k, b) or [None, '?'])[1]
            return {k: get(k) for k in ('vgpr_count', 'sgpr_count', 'vgpr_spill_count', 'sgpr_spill_count',
                                        'private_segment_fixed_size')}
    return {}


def loops(asm, name):
    lines = asm.split('\n')
    start = next(i for i, l in enumerate(lines) if l.endswith('>:') and name in l)
    end = next((i for i in range(start + 1, len(lines)) if re.match(r'^[0-9a-f]+ <', lines[i])), len(lines))
    ins = []
    for l in lines[start + 1:end]:
        m = re.match(r'^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):[^<]*(?:<[^+]*\+0x([0-9a-f]+)>)?', l)
        if m:
            ins.append((int(m.group(3), 16), m.group(1), int(m.group(4), 16) if m.group(4) else None))
    base = ins[0][0]
    at = {a - base: i for i, (a, _, _) in enumerate(ins)}
    out = []
    for i, (a, op, t) in enumerate(ins):
        if (op.startswith('s_cbranch') or op == 's_branch') and t is not None and t < a - base and t in at:
            seg = ins[at[t]:i + 1]
            c = collections.Counter('mfma' if 'mfma' in o else '_'.join(o.split('_')[:2]) for _, o, _ in seg)
            if c['mfma']:
                out.append((at[t], i, len(seg), c))
    return lines[start].split('<')[1].rstrip('>:'), len(ins), out


def main():
    obj, name = sys.argv[1], sys.argv[2]
    with tempfile.TemporaryDirectory() as tmp:
        asm, notes = disassemble(obj, tmp)
    full, n, found = loops(asm, name)
    print(full)
    print('instructions %d; %s' % (n, kernel_meta(notes, name)))
    for j, i, ln, c in found:
        keys = ('mfma', 'ds_read', 'buffer_load', 'scratch_store', 'scratch_load', 's_waitcnt', 'v_readfirstlane')
        extra = ', '.join('%s %d' % (k, c[k]) for k in keys if c[k])
        print('  loop [%d..%d] %d instructions: %s' % (j, i, ln, extra))


if __name__ == '__main__':
    main()
