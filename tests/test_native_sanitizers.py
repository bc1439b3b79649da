"""Host-code sanitizer runs.

The host C++ twins of NMS and RoI pooling (mx_rcnn_amd/csrc/host_ops.h, linked into the
extension through bindings.cpp) are compiled into tests/native/host_ops_test.cpp twice --
under AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer -- and run on
the CPU.  The driver checks them against independent oracles, bitwise repeatability and the
concurrent-range contract used by at::parallel_for.  GPU-side sanitizers (device ASan,
xnack+) are not available on this pool, so device kernels are covered by the fp32-oracle
numerics tests in test_kernels.py instead.
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, 'native', 'host_ops_test.cpp')
INC = os.path.join(os.path.dirname(HERE), 'mx_rcnn_amd', 'csrc')

SANITIZERS = {
    'asan_ubsan': ['-fsanitize=address,undefined', '-fsanitize=float-cast-overflow', '-fno-sanitize-recover=all',
                   '-fno-omit-frame-pointer'],
    'tsan': ['-fsanitize=thread'],
}


@pytest.mark.parametrize('kind', sorted(SANITIZERS))
def test_host_ops_under_sanitizer(kind, tmp_path):
    cxx = shutil.which(os.environ.get('CXX', 'g++'))
    if cxx is None:
        pytest.skip('no host C++ compiler')
    exe = str(tmp_path / ('host_ops_' + kind))
    cmd = [cxx, '-std=c++17', '-O1', '-g', '-pthread', '-I', INC, SRC, '-o', exe] + SANITIZERS[kind]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:verify_asan_link_order=0',
               UBSAN_OPTIONS='print_stacktrace=1', TSAN_OPTIONS='halt_on_error=1')
    r = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300, env=env)
    assert r.returncode == 0 and 'host_ops_test OK' in r.stdout, r.stdout
