"""Host-side sanitizer run (SURVEY §5 race detection / sanitizers): the C++
host codec and event loop rebuilt with ASan + UBSan (codec suites: parity,
golden vectors, hypothesis fuzz; loop and client suites), then the event
loop rebuilt with ThreadSanitizer under the loop / client / fault-injection
suites — all in a child process (tools/sanitize_host.sh)."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _have_asan():
    if shutil.which('gcc') is None or shutil.which('g++') is None:
        return False
    lib = subprocess.run(['gcc', '-print-file-name=libasan.so'],
                         capture_output=True, text=True).stdout.strip()
    return os.path.isabs(lib) and os.path.exists(lib)


@pytest.mark.slow
@pytest.mark.skipif(not _have_asan(), reason='no gcc ASan runtime')
def test_host_codec_under_asan_ubsan():
    env = dict(os.environ)
    env.pop('ZKMI_HOST_CODEC', None)
    r = subprocess.run(['bash', os.path.join(ROOT, 'tools',
                                             'sanitize_host.sh')],
                       cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count(' passed') >= 2        # ASan/UBSan + TSan runs
