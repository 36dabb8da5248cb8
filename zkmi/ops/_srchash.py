"""Source hashes of the native artefacts.

``tools/build_native.py`` stamps every artefact it builds with the hash of
the sources (and flags) it was built from: the HIP kernel library carries
it as a symbol (``zkmi_hip_src_hash``), the others in a ``<artefact>.srchash``
file next to them.  A build is redone whenever the stamp differs from the
tree's hash (never by file age), and :func:`zkmi.ops._lib.lib` refuses to
load a kernel library whose embedded hash is not the hash of the kernel
sources in this tree — so a GPU run always tests code compiled from the
sources it ships with.
"""

import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))
KDIR = os.path.join(ROOT, 'csrc', 'kernels')

ARCH = 'gfx950'                  # MI355X only
HIP_FLAGS = ['--offload-arch=' + ARCH, '-O3', '-fPIC', '-std=c++17',
             '-Wno-unused-result', '-Wno-unused-value', '-munsafe-fp-atomics']


def files_hash(files, extra=''):
    """16 hex digits of sha256 over (name, bytes) of ``files`` + ``extra``."""
    h = hashlib.sha256(extra.encode())
    for f in sorted(files):
        h.update(os.path.relpath(f, ROOT).encode() + b'\0')
        with open(f, 'rb') as fh:
            h.update(fh.read())
        h.update(b'\0')
    return h.hexdigest()[:16]


def hip_sources():
    return sorted(os.path.join(KDIR, f) for f in os.listdir(KDIR)
                  if f.endswith('.hip') or f.endswith('.h'))


def hip_hash():
    """Hash of the kernel library's sources and compile flags."""
    return files_hash(hip_sources(), ' '.join(HIP_FLAGS))


def read_stamp(artefact):
    try:
        with open(artefact + '.srchash') as f:
            return f.read().strip()
    except OSError:
        return None


def write_stamp(artefact, value):
    with open(artefact + '.srchash', 'w') as f:
        f.write(value + '\n')
