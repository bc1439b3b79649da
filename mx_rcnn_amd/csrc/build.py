"""In-tree build of the gfx950 extension ``mx_rcnn_amd/_C*.so``.

Explicit hipcc pipeline (no hipify, no JIT cache): every ``hip/*.hip`` is compiled with
``hipcc --offload-arch=gfx950`` into a PIC object, ``bindings.cpp`` (host-only glue)
with the host compiler against the PyTorch headers, and everything is linked into one
shared object next to the package so it travels with the repo snapshot to the GPU box.
Incremental: an object is rebuilt only when its source or a header is newer.

Usage: ``python -m mx_rcnn_amd.csrc.build [--force] [--jobs N] [--debug]``
"""
import argparse
import glob
import os
import re
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
BUILD = os.path.join(HERE, '_build')
ROCM = os.environ.get('ROCM_PATH', '/opt/rocm')
ARCH = os.environ.get('MXR_OFFLOAD_ARCH', 'gfx950')


def _torch_paths():
    import torch
    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, 'include'), os.path.join(root, 'include', 'torch', 'csrc', 'api', 'include')]
    return root, inc, os.path.join(root, 'lib'), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def ext_path():
    """The in-tree extension, or MXR_EXT_OUT when set (a staging path: link elsewhere while the
    in-tree .so is in use, then copy it in)."""
    if os.environ.get('MXR_EXT_OUT'):
        return os.environ['MXR_EXT_OUT']
    suffix = sysconfig.get_config_var('EXT_SUFFIX') or '.so'
    return os.path.join(PKG, '_C' + suffix)


def _newer(src_list, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_list)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError('build step failed:\n%s\n%s' % (' '.join(cmd), r.stdout))
    return r.stdout


_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _local_deps(src, seen=None):
    """The in-tree headers ``src`` includes, transitively (quoted includes resolved next to the
    including file, then in csrc/ and csrc/hip/): an object rebuilds only when one of ITS headers
    changes (a conv-body edit no longer rebuilds every kernel file)."""
    seen = set() if seen is None else seen
    try:
        text = open(src).read()
    except OSError:
        return seen
    for name in _INC.findall(text):
        for d in (os.path.dirname(src), HERE, os.path.join(HERE, 'hip')):
            path = os.path.normpath(os.path.join(d, name))
            if os.path.exists(path):
                if path not in seen:
                    seen.add(path)
                    _local_deps(path, seen)
                break
    return seen


def build(force=False, jobs=None, debug=False, verbose=False):
    os.makedirs(BUILD, exist_ok=True)
    troot, tinc, tlib, abi = _torch_paths()
    hipcc = os.path.join(ROCM, 'bin', 'hipcc')
    opt = ['-O0', '-g'] if debug else ['-O3']
    hip_flags = opt + ['--offload-arch=%s' % ARCH, '-fPIC', '-std=c++17', '-ffp-contract=off',
                       '-D_GLIBCXX_USE_CXX11_ABI=%d' % abi, '-I', HERE, '-I', os.path.join(HERE, 'hip')]
    if os.environ.get('MXR_SYNC_DEBUG'):
        hip_flags.append('-DMXR_SYNC_DEBUG=1')
    jobs_list = []
    objs = []
    for src in sorted(glob.glob(os.path.join(HERE, 'hip', '*.hip'))):
        obj = os.path.join(BUILD, os.path.basename(src) + '.o')
        objs.append(obj)
        if force or _newer([src] + sorted(_local_deps(src)), obj):
            jobs_list.append([hipcc] + hip_flags + ['-c', src, '-o', obj])
    py_inc = sysconfig.get_paths()['include']
    glue = os.path.join(HERE, 'bindings.cpp')
    glue_obj = os.path.join(BUILD, 'bindings.o')
    objs.append(glue_obj)
    if force or _newer([glue] + sorted(_local_deps(glue)), glue_obj):
        cxx = os.environ.get('CXX', 'g++')
        flags = opt + ['-fPIC', '-std=c++17', '-D__HIP_PLATFORM_AMD__=1', '-DUSE_ROCM=1',
                       '-DTORCH_EXTENSION_NAME=_C', '-DTORCH_API_INCLUDE_EXTENSION_H',
                       '-D_GLIBCXX_USE_CXX11_ABI=%d' % abi, '-I', HERE, '-I', os.path.join(ROCM, 'include'),
                       '-I', py_inc] + sum([['-I', p] for p in tinc], []) + ['-w']
        jobs_list.append([cxx] + flags + ['-c', glue, '-o', glue_obj])
    n = jobs or min(8, max(1, len(jobs_list)))
    with ThreadPoolExecutor(n) as ex:
        for out in ex.map(_run, jobs_list):
            if verbose and out.strip():
                print(out)
    target = ext_path()
    if force or jobs_list or not os.path.exists(target) or _newer(objs, target):
        link = ['g++', '-shared', '-o', target] + objs + [
            '-L', tlib, '-Wl,-rpath,' + tlib, '-lc10', '-lc10_hip', '-ltorch', '-ltorch_cpu', '-ltorch_hip',
            '-ltorch_python', '-lamdhip64']
        _run(link)
    return target


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('--jobs', type=int, default=None)
    ap.add_argument('--debug', action='store_true')
    ap.add_argument('-v', '--verbose', action='store_true')
    a = ap.parse_args()
    print(build(force=a.force, jobs=a.jobs, debug=a.debug, verbose=a.verbose))


if __name__ == '__main__':
    sys.exit(main())
