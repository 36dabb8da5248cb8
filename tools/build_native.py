"""Build the native parts of zkmi in-tree.

* ``zkmi/ops/libzkmi_hip.so`` — the HIP/CDNA4 batch codec kernels
  (csrc/kernels/*.hip), compiled with ``hipcc --offload-arch=gfx950``.  It
  links libamdhip64.so.7, which resolves to the copy torch already loaded
  (same soname), so torch and zkmi share one HIP runtime.
* ``zkmi/_zkhost*.so`` — the C++ host codec for the interactive path
  (csrc/host), a CPython extension (no torch headers).

Usage: ``python tools/build_native.py [--hip-only|--host-only|--sanitize]
[-j N]``.
Objects are cached under ``build/``.  Every artefact is stamped with the
hash of the sources and flags it was built from (``zkmi/ops/_srchash.py``)
and rebuilt whenever that differs from the tree's hash — never by file age,
so prebuilt binaries from another tree are never reused.  The kernel library
embeds its hash (``zkmi_hip_src_hash``), which the loader checks.
"""

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from zkmi.ops import _srchash as SH  # noqa: E402
KDIR = os.path.join(ROOT, 'csrc', 'kernels')
HDIR = os.path.join(ROOT, 'csrc', 'host')
BDIR = os.path.join(ROOT, 'build')
HIP_SO = os.path.join(ROOT, 'zkmi', 'ops', 'libzkmi_hip.so')
ARCH = SH.ARCH
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True)
    if r.returncode != 0:
        sys.stderr.write(' '.join(cmd) + '\n' + r.stdout)
        raise RuntimeError('command failed: %s' % cmd[0])
    return r.stdout


def _stale(out, deps, extra=''):
    """(rebuild needed, hash): ``out`` is missing or its stamp is not the
    hash of ``deps`` + ``extra``."""
    h = SH.files_hash(deps, extra)
    return (not os.path.exists(out) or SH.read_stamp(out) != h), h


def _stamped(out, h):
    SH.write_stamp(out, h)
    return out


def build_hip(jobs=4):
    os.makedirs(BDIR, exist_ok=True)
    srcs = sorted(f for f in os.listdir(KDIR) if f.endswith('.hip'))
    hdrs = [os.path.join(KDIR, f) for f in os.listdir(KDIR)
            if f.endswith('.h')]
    flags = SH.HIP_FLAGS
    objs = []
    todo = []
    for s in srcs:
        src = os.path.join(KDIR, s)
        obj = os.path.join(BDIR, s.replace('.hip', '.o'))
        objs.append(obj)
        stale, h = _stale(obj, [src] + hdrs, ' '.join(flags))
        if stale:
            todo.append((obj, h, [HIPCC] + flags + ['-c', src, '-o', obj]))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda t: (_run(t[2]), _stamped(t[0], t[1])), todo))
    full = SH.hip_hash()

    def embedded():
        # the hash string the library itself carries (a library copied over
        # the built one keeps a matching stamp file but not this)
        with open(HIP_SO, 'rb') as f:
            return full.encode() in f.read()
    if todo or SH.read_stamp(HIP_SO) != full or not os.path.exists(HIP_SO) \
            or not embedded():
        # the library carries the hash of the sources it was built from
        stamp_src = os.path.join(BDIR, 'zkmi_stamp.cpp')
        with open(stamp_src, 'w') as f:
            f.write('extern "C" const char *zkmi_hip_src_hash(void) '
                    '{ return "%s"; }\n' % full)
        stamp_obj = os.path.join(BDIR, 'zkmi_stamp.o')
        _run(['g++', '-O2', '-fPIC', '-c', stamp_src, '-o', stamp_obj])
        _run([HIPCC, '--offload-arch=' + ARCH, '-shared', '-fPIC', '-o',
              HIP_SO] + objs + [stamp_obj])
        _stamped(HIP_SO, full)
    return HIP_SO


TORCH_SO = os.path.join(ROOT, 'zkmi', 'ops', 'libzkmi_torch.so')
TDIR = os.path.join(ROOT, 'csrc', 'torch')


def build_torch_ops():
    """``zkmi/ops/libzkmi_torch.so``: the TORCH_LIBRARY(zkmi, ...) operator
    library (csrc/torch/zkmi_ops.cpp) over libzkmi_hip.so, loaded with
    ``torch.ops.load_library`` (torch.ops.zkmi.*).  Built with the host
    compiler against torch's headers; the kernels stay in libzkmi_hip.so
    (found through the rpath)."""
    import torch
    src = os.path.join(TDIR, 'zkmi_ops.cpp')
    deps = [src, os.path.join(KDIR, 'zk_abi.h')]
    stale, h = _stale(TORCH_SO, deps, torch.__version__)
    if not stale:
        return TORCH_SO
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, 'include'),
           os.path.join(tdir, 'include', 'torch', 'csrc', 'api', 'include'),
           '/opt/rocm/include']
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    _run(['g++', '-O2', '-fPIC', '-shared', '-std=c++17', '-Wall',
          '-Wno-unused-function', '-D__HIP_PLATFORM_AMD__=1', '-DUSE_ROCM=1',
          '-D_GLIBCXX_USE_CXX11_ABI=%d' % abi] +
         ['-I' + i for i in inc] +
         [src, '-o', TORCH_SO, '-L' + os.path.join(tdir, 'lib'),
          '-L' + os.path.dirname(HIP_SO), '-lzkmi_hip', '-lc10', '-lc10_hip',
          '-ltorch_cpu', '-Wl,-rpath,$ORIGIN',
          '-Wl,-rpath,' + os.path.join(tdir, 'lib')])
    return _stamped(TORCH_SO, h)


def host_so_path():
    return _ext_path('_zkhost')


def _ext_path(name):
    suffix = sysconfig.get_config_var('EXT_SUFFIX') or '.so'
    return os.path.join(ROOT, 'zkmi', name + suffix)


# CPython extensions built from csrc/host: module name -> source
HOST_EXTS = {'_zkhost': 'zk_host_codec.cpp',     # Jute host codec
             '_zkloop': 'zk_loop.cpp',           # epoll event loop
             '_zkwatch': 'zk_watch.cpp',         # watch-event engine
             '_zkfsm': 'zk_fsm.cpp',             # FSM runtime
             # session / connection / client machines
             '_zkmach': 'zk_machines.cpp'}


FAST_SERVER = os.path.join(ROOT, 'zkmi', 'bin', 'zk_fastserver')


def build_fastserver():
    """The native benchmark server (csrc/host/zk_fastserver.cpp), a plain
    executable: zkmi/server/fast.py runs it as a child process."""
    src = os.path.join(HDIR, 'zk_fastserver.cpp')
    os.makedirs(os.path.dirname(FAST_SERVER), exist_ok=True)
    stale, h = _stale(FAST_SERVER, [src])
    if stale:
        _run(['g++', '-O3', '-std=c++17', '-Wall', '-Wextra', src, '-o',
              FAST_SERVER, '-lpthread'])
        _stamped(FAST_SERVER, h)
    return FAST_SERVER


def build_host():
    outs = [build_fastserver()]
    inc = sysconfig.get_paths()['include']
    for name, src in HOST_EXTS.items():
        src = os.path.join(HDIR, src)
        out = _ext_path(name)
        stale, h = _stale(out, [src])
        if stale:
            _run(['g++', '-O3', '-fPIC', '-shared', '-std=c++17', '-Wall',
                  '-Wextra', '-Wno-missing-field-initializers',
                  '-Wno-cast-function-type', '-fno-strict-aliasing',
                  '-I' + inc, src, '-o', out])
            _stamped(out, h)
        outs.append(out)
    return outs


SANITIZE_DIR = os.path.join(BDIR, 'sanitize')


def build_host_sanitized():
    """The host extensions (codec and event loop) built with
    AddressSanitizer + UndefinedBehaviorSanitizer (host code only — GPU
    sanitizers are not used).  Load them with ``ZKMI_HOST_CODEC_PATH`` /
    ``ZKMI_NATIVE_LOOP_PATH`` and the sanitizer runtimes preloaded (see
    tools/sanitize_host.sh).  Returns the two paths."""
    os.makedirs(SANITIZE_DIR, exist_ok=True)
    suffix = sysconfig.get_config_var('EXT_SUFFIX') or '.so'
    inc = sysconfig.get_paths()['include']
    outs = []
    for name, src in HOST_EXTS.items():
        src = os.path.join(HDIR, src)
        out = os.path.join(SANITIZE_DIR, name + suffix)
        stale, h = _stale(out, [src], 'asan')
        if stale:
            _run(['g++', '-O1', '-g', '-fPIC', '-shared', '-std=c++17',
                  '-Wall', '-fno-strict-aliasing', '-fno-omit-frame-pointer',
                  '-fsanitize=address,undefined', '-fno-sanitize-recover=all',
                  '-I' + inc, src, '-o', out])
            _stamped(out, h)
        outs.append(out)
    return outs


TSAN_DIR = os.path.join(BDIR, 'tsan')


def build_loop_tsan():
    """The native event loop (the only threaded host code) built with
    ThreadSanitizer.  CPython's GIL is a pthread mutex/condvar pair, which
    TSan intercepts, so GIL hand-offs count as synchronisation and only
    genuinely unsynchronised accesses are reported."""
    os.makedirs(TSAN_DIR, exist_ok=True)
    suffix = sysconfig.get_config_var('EXT_SUFFIX') or '.so'
    src = os.path.join(HDIR, HOST_EXTS['_zkloop'])
    out = os.path.join(TSAN_DIR, '_zkloop' + suffix)
    stale, h = _stale(out, [src], 'tsan')
    if stale:
        inc = sysconfig.get_paths()['include']
        _run(['g++', '-O1', '-g', '-fPIC', '-shared', '-std=c++17', '-Wall',
              '-fsanitize=thread', '-I' + inc, src, '-o', out])
        _stamped(out, h)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--hip-only', action='store_true')
    ap.add_argument('--host-only', action='store_true')
    ap.add_argument('--sanitize', action='store_true',
                    help='build only the ASan/UBSan host codec')
    ap.add_argument('--tsan', action='store_true',
                    help='build only the ThreadSanitizer event loop')
    ap.add_argument('-j', type=int, default=4)
    a = ap.parse_args()
    if a.tsan:
        print(build_loop_tsan())
        return
    if a.sanitize:
        print(' '.join(build_host_sanitized()))
        return
    if not a.host_only:
        print(build_hip(a.j))
        print(build_torch_ops())
    if not a.hip_only:
        print(build_host())


if __name__ == '__main__':
    main()
