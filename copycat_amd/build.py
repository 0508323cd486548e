"""In-tree build of the native libraries (no JIT cache: the .so files travel with the repo snapshot).

  libcopycat_apply.so     hipcc --offload-arch=gfx950: the engine (HIP kernels + C-ABI)
  libcopycat_workload.so  g++: synthetic committed-command stream generators for benches/tests
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)

ENGINE_SRCS = ["engine.hip", "map_big.hip", "partition.hip", "partition_ext.hip", "apply_value.hip", "value_path.hip", "apply_map.hip", "apply_map_hot.hip", "apply_coord.hip", "events.hip", "quorum.hip", "close.hip", "map_wide.hip", "live.hip", "manager.hip", "retained.hip", "host_path.hip", "map_small.hip", "map_cv.hip", "map_clear.hip", "wire.cpp", "split.cpp"]
ENGINE_HDRS = ["common.h", "engine_internal.h", "engine_state.h", "map_ops.h", "java_hashmap.h", "small_jhm.h", "jhm_tree.h", "big_jhm.h"]
ENGINE_SO = os.path.join(HERE, "libcopycat_apply.so")
WORKLOAD_SO = os.path.join(HERE, "libcopycat_workload.so")
ARCH = os.environ.get("CC_OFFLOAD_ARCH", "gfx950")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build failed: {' '.join(cmd)}")


def build_engine(force=False):
    deps = [os.path.join(CSRC, f) for f in ENGINE_SRCS + ENGINE_HDRS] + [os.path.join(ROOT, "include", "copycat_apply.h")]
    if force or _stale(ENGINE_SO, deps):
        hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
        flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall"]
        objdir = os.path.join(HERE, "build_obj")
        os.makedirs(objdir, exist_ok=True)
        objs = [os.path.join(objdir, os.path.splitext(f)[0] + ".o") for f in ENGINE_SRCS]
        # one hipcc per translation unit, in parallel (every kernel is launched from the unit that defines it)
        from concurrent.futures import ThreadPoolExecutor

        jobs = max(1, min(len(ENGINE_SRCS), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1)), 16))
        with ThreadPoolExecutor(jobs) as ex:
            list(ex.map(lambda so: _run([hipcc, *flags, "-c", so[0], "-o", so[1]]), zip(ENGINE_SRCS, objs)))
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", ENGINE_SO])
    return ENGINE_SO


def build_variant(out_path, defines, tag):
    """A diagnostics / A-B build of the engine with extra -D flags (object files under build_obj/<tag>)."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall"] + [f"-D{d}" for d in defines]
    objdir = os.path.join(HERE, "build_obj", tag)
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.splitext(f)[0] + ".o") for f in ENGINE_SRCS]
    from concurrent.futures import ThreadPoolExecutor

    jobs = max(1, min(len(ENGINE_SRCS), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1)), 16))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(lambda so: _run([hipcc, *flags, "-c", so[0], "-o", so[1]]), zip(ENGINE_SRCS, objs)))
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out_path])
    return out_path


def build_workload(force=False):
    src = os.path.join(CSRC, "workload.cpp")
    if force or _stale(WORKLOAD_SO, [src]):
        _run([os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-pthread", "workload.cpp",
              "-o", WORKLOAD_SO])
    return WORKLOAD_SO


def build_all(force=False):
    return build_engine(force), build_workload(force)


if __name__ == "__main__":
    print(build_all(force="--force" in sys.argv))
