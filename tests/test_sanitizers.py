"""Host sanitizer build (SURVEY §5 "Race detection / sanitizers").

`make -C real-time-voice-cloning_amd/csrc asan` builds the library's host C++ -- the libwavernn
.bin reader (binfile.cpp, which parses user files) and the f64 post-processing loops
(host_post.cpp) -- with AddressSanitizer + UndefinedBehaviorSanitizer, no HIP, as
build/asan/libwavernn_host_asan.so. This test runs the host tests against that library in a
child process (WRNN_LIB / WRNN_HOST_ONLY; the ASan runtime preloaded first, leak checking off
for the Python interpreter) and requires a clean run: every .bin round trip, every corrupt-file
refusal (tests/test_bin_corrupt.py: truncations, lengths past the file, out-of-range and
negative-in-int8 column groups, zero-row layers, 200 random corruptions) and every
post-processing case, with no sanitizer report. A canary first checks the sanitizer is live: an
output buffer one element short must be reported.
"""
import os
import subprocess
import sys

import pytest

from conftest import PKG, REPO

CSRC = os.path.join(PKG, 'csrc')
ASAN_LIB = os.path.join(CSRC, 'build', 'asan', 'libwavernn_host_asan.so')
HOST_TESTS = ['tests/test_bin_corrupt.py', 'tests/test_libwavernn.py', 'tests/test_host_post.py']


def _env():
    libasan = subprocess.run(['gcc', '-print-file-name=libasan.so'], capture_output=True,
                             text=True, check=True).stdout.strip()
    env = dict(os.environ)
    pre = env.get('LD_PRELOAD', '')
    env.update(WRNN_LIB=ASAN_LIB, WRNN_HOST_ONLY='1',
               LD_PRELOAD=libasan + (':' + pre if pre else ''),  # the ASan runtime must be first
               ASAN_OPTIONS='detect_leaks=0:abort_on_error=1',
               UBSAN_OPTIONS='halt_on_error=1:print_stacktrace=1', PYTHONPATH=PKG + ':' + REPO)
    return env


@pytest.fixture(scope='module')
def asan_lib():
    r = subprocess.run(['make', '-C', CSRC, 'asan'], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail('make asan failed:\n' + r.stdout[-2000:] + r.stderr[-2000:])
    return ASAN_LIB


CANARY = r'''
import numpy as np
from wavernn_amd import _abi
lib = _abi.load_library()
assert b'sanitizer' in lib.wrnn_version(), lib.wrnn_version()
nf, S, ov = 3, 40, 10
labels = np.zeros((nf, S), np.int16)
samp = np.zeros(512); fin = np.ones(ov); fout = np.ones(ov)
regions = np.empty((nf + 1) * ov - 1)  # one element short
lib.wrnn_post_overlaps(labels.ctypes.data, nf, S, ov, samp.ctypes.data, 512, fin.ctypes.data,
                       fout.ctypes.data, regions.ctypes.data)
print('NOT DETECTED')
'''


def test_sanitizer_is_live(asan_lib):
    r = subprocess.run([sys.executable, '-c', CANARY], env=_env(), capture_output=True, text=True,
                       cwd=REPO, timeout=300)
    assert 'NOT DETECTED' not in r.stdout
    assert 'AddressSanitizer: heap-buffer-overflow' in r.stderr, r.stderr[-3000:]


def test_host_tests_clean_under_asan_ubsan(asan_lib):
    r = subprocess.run([sys.executable, '-m', 'pytest', '-q', '-p', 'no:cacheprovider', *HOST_TESTS],
                       env=_env(), capture_output=True, text=True, cwd=REPO, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert 'AddressSanitizer' not in out and 'runtime error:' not in out, out[-4000:]
    assert ' passed' in r.stdout
