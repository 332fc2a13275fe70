"""Build the native library ``handyrl_amd/_lib/libhrl.so`` with hipcc for gfx950.

Each ``csrc/*.hip`` translation unit is compiled to an object in parallel,
then linked into one shared library exporting the C ABI of ``include/*.h``.
The library is built in-tree so it travels with the repository snapshot to
the GPU box (it is git-ignored, not gpurun-ignored).

    python -m handyrl_amd.build [--force]
"""

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'handyrl_amd')
CSRC = os.path.join(PKG, 'csrc')
INCLUDE = os.path.join(ROOT, 'include')
OUT_DIR = os.path.join(PKG, '_lib')
OBJ_DIR = os.path.join(ROOT, 'build', 'obj')
LIB = os.path.join(OUT_DIR, 'libhrl.so')
ARCH = os.environ.get('HRL_OFFLOAD_ARCH', 'gfx950')

# -ffp-contract=off: the scans and loss kernels reproduce the reference's
# float32 operation order exactly; no a*b+c contraction into FMA.
HIPCC_FLAGS = ['--offload-arch=%s' % ARCH, '-O3', '-std=c++17', '-fPIC', '-ffp-contract=off',
               '-Wall', '-Wno-unused-function', '-I', INCLUDE]


def hipcc():
    exe = shutil.which('hipcc') or '/opt/rocm/bin/hipcc'
    if not os.path.exists(exe):
        raise RuntimeError('hipcc not found: the HIP library cannot be built')
    return exe


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.hip'))


def _obj_of(src):
    return os.path.join(OBJ_DIR, os.path.basename(src) + '.o')


def up_to_date():
    """The library is newer than every object and every object newer than its source and the headers (a source
    edited while a build ran leaves its object older than the source, so the next build recompiles it)."""
    if not os.path.exists(LIB):
        return False
    hdrs = [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE)]
    hdrs += [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.h')]
    deps = max(os.path.getmtime(h) for h in hdrs)
    lib_t = os.path.getmtime(LIB)
    for src in sources():
        obj = _obj_of(src)
        if not os.path.exists(obj):
            return False
        t = os.path.getmtime(obj)
        if t < max(deps, os.path.getmtime(src)) or t > lib_t:
            return False
    return True


def _compile(src):
    obj = _obj_of(src)
    hdrs = [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE)]
    hdrs += [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.h')]
    hdr_mtime = max(os.path.getmtime(h) for h in hdrs)
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime):
        return obj
    cmd = [hipcc()] + HIPCC_FLAGS + ['-c', src, '-o', obj]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError('hipcc failed for %s:\n%s\n%s' % (src, ' '.join(cmd), res.stderr))
    return obj


def build(force=False, verbose=True):
    """Compile every HIP source for gfx950 and link libhrl.so (skips if up to date)."""
    if not force and up_to_date():
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    os.makedirs(OBJ_DIR, exist_ok=True)
    if force:
        for f in os.listdir(OBJ_DIR):
            os.remove(os.path.join(OBJ_DIR, f))
    srcs = sources()
    workers = min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(workers) as ex:
        objs = list(ex.map(_compile, srcs))
    tmp = LIB + '.tmp'
    cmd = [hipcc(), '--offload-arch=%s' % ARCH, '-shared', '-fPIC', '-o', tmp] + objs
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError('link failed:\n%s\n%s' % (' '.join(cmd), res.stderr))
    os.replace(tmp, LIB)
    if verbose:
        print('built %s from %d sources' % (LIB, len(srcs)))
    return LIB


if __name__ == '__main__':
    build(force='--force' in sys.argv)
