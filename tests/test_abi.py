"""The C-ABI library: loads, exports every symbol include/footsies.h declares, struct layouts
agree between C (gcc on the header) and the ctypes mirror, and creation without a GPU fails
loudly with a message instead of falling back to anything."""
import ctypes as C
import os
import re
import subprocess

import pytest

from footsies_gym_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "footsies.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(fs_[a-z_0-9]+)\(", text, re.M)))


@pytest.fixture(scope="module")
def lib():
    import torch  # noqa: F401 -- first, as _lib.lib() does: one HIP runtime in the process
    from footsies_gym_amd import build
    build.build()
    return C.CDLL(build.LIB)


def test_exports_every_declared_symbol(lib):
    names = declared_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
        assert n in _abi.LIB_FUNCTIONS, "ctypes binding misses %s" % n
    assert set(_abi.LIB_FUNCTIONS) == set(names)


def test_abi_version(lib):
    lib.fs_abi_version.restype = C.c_int
    assert lib.fs_abi_version() == _abi.FS_ABI_VERSION


def _c_layout(tmp_path):
    structs = {"fs_config": _abi.fs_config, "fs_outputs": _abi.fs_outputs, "fs_env_state": _abi.fs_env_state,
               "fs_fighter_state": _abi.fs_fighter_state, "fs_arena_state": _abi.fs_arena_state,
               "fs_policy": _abi.fs_policy, "fs_mlp": _abi.fs_mlp}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "footsies.h"', "int main(void){"]
    for s, cls in structs.items():
        lines.append('printf("%s size %%zu\\n", sizeof(%s));' % (s, s))
        for f, _ in cls._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (s, f, s, f))
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    return structs, dict(line.rsplit(" ", 1) for line in out.strip().splitlines())


def test_struct_layouts_match_ctypes(tmp_path):
    structs, c = _c_layout(tmp_path)
    for s, cls in structs.items():
        assert int(c["%s size" % s]) == C.sizeof(cls), s
        for f, _ in cls._fields_:
            assert int(c["%s.%s" % (s, f)]) == getattr(cls, f).offset, (s, f)


def test_create_without_gpu_fails_loudly(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    lib.fs_create.argtypes = [C.POINTER(_abi.fs_config), C.POINTER(C.c_void_p)]
    lib.fs_last_error.restype = C.c_char_p
    lib.fs_last_error.argtypes = [C.c_void_p]
    h = C.c_void_p()
    cfg = _abi.fs_config(num_envs=4)
    rc = lib.fs_create(C.byref(cfg), C.byref(h))
    assert rc == _abi.FS_E_DEVICE
    assert not h.value
    assert lib.fs_last_error(None)


def test_invalid_configs_rejected(lib):
    lib.fs_create.argtypes = [C.POINTER(_abi.fs_config), C.POINTER(C.c_void_p)]
    h = C.c_void_p()
    for kw, code in [({"num_envs": 0}, _abi.FS_E_INVALID), ({"num_envs": 4, "p2_mode": 9}, _abi.FS_E_INVALID),
                     ({"num_envs": 4, "frame_delay": -1}, _abi.FS_E_INVALID),
                     ({"num_envs": 4, "frame_delay": _abi.FS_MAX_FRAME_DELAY + 1}, _abi.FS_E_INVALID),
                     ({"num_envs": 4, "float_mode": 7}, _abi.FS_E_INVALID)]:
        assert lib.fs_create(C.byref(_abi.fs_config(**kw)), C.byref(h)) == code, kw


def test_simulator_requires_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from footsies_gym_amd.simulator import FootsiesSim
    with pytest.raises(RuntimeError):
        FootsiesSim(8)


def test_step_kernel_name_needs_a_handle(lib):
    """fs_step_kernel (the kernel a step call launches, for profiles and the roofline line) answers
    NULL without a handle; the names themselves are checked on the GPU (test_gpu_api.py)."""
    f = lib.fs_step_kernel
    f.restype, f.argtypes = _abi.LIB_FUNCTIONS["fs_step_kernel"]
    assert f(None, 1, 0) is None


def test_one_hip_runtime_per_process():
    """The binding loads torch before libfootsies.so, so the library's libamdhip64.so.7 entry binds
    to torch's runtime: one HIP and one HSA runtime per process.  Loaded the other way round the
    process maps /opt/rocm's runtimes beside torch's, and fs_create found no device on the MI355X
    box (profiles/r05q_lib_before_torch.log, r05p_lib_before_torch_test.log)."""
    import subprocess
    import sys
    code = ("from footsies_gym_amd._lib import lib; lib(); import torch; "
            "m = {l.split()[-1] for l in open('/proc/self/maps') if 'amdhip64' in l or 'hsa-runtime64' in l}; "
            "print(sum('amdhip64' in x for x in m), sum('hsa-runtime64' in x for x in m))")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split()[-2:] == ["1", "1"], r.stdout


def test_ppo_grad_runs_argument_checks():
    """fs_ppo_grad_runs rejects on the host, before any launch: no runs, n_runs <= 0, a run shift
    outside [0, 30], a table shorter than one run (no GPU needed: nothing is launched)."""
    from footsies_gym_amd._lib import lib as load
    L = load()
    rows = (C.c_float * 48)()
    runs = (C.c_int64 * 4)()
    mlp = _abi.fs_mlp()
    ws = (C.c_uint8 * 16)()

    def call(runs_ptr, n_rows, n_runs, shift):
        return L.fs_ppo_grad_runs(C.cast(rows, C.c_void_p), n_rows, runs_ptr, n_runs, shift, C.byref(mlp),
                                  C.byref(mlp), 0.2, 0.5, 0.01, C.cast(rows, C.c_void_p), C.cast(rows, C.c_void_p),
                                  C.cast(ws, C.c_void_p), 16, None, _abi.FS_PPO_SPLIT_BF16)
    rp = C.cast(runs, C.c_void_p)
    for args in ((None, 4, 4, 0), (rp, 4, 0, 0), (rp, 4, 4, -1), (rp, 4, 4, 31), (rp, 4, 4, 3), (rp, 0, 4, 0)):
        assert call(*args) == _abi.FS_E_INVALID, args


def _run(code):
    import sys
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def test_second_runtime_is_named_in_the_create_error():
    """A second HSA runtime image mapped beside the one libfootsies bound to (what loading the library
    before torch did on the MI355X box, profiles/r05q_lib_before_torch.log): fs_runtime_images lists
    both, and fs_create -- which then sees no device -- returns FS_E_RUNTIME naming both paths instead
    of "no ROCm-capable device".  Needs two distinct runtime files (torch's bundled copy and
    /opt/rocm's); skipped where the image has one."""
    import glob
    import torch
    tdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    rocm = sorted(glob.glob("/opt/rocm/lib/libhsa-runtime64.so.1.*"))
    if not os.path.exists(os.path.join(tdir, "libhsa-runtime64.so")) or not rocm:
        pytest.skip("one HSA runtime in this image")
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible: fs_create would succeed on the bound runtime's device list")
    out = _run("import ctypes as C, torch\n"
               "C.CDLL(%r)\n"
               "from footsies_gym_amd import _lib, _abi\n"
               "L = _lib.lib()\n"
               "print(repr(_lib.runtime_images()))\n"
               "h = C.c_void_p()\n"
               "print(L.fs_create(C.byref(_abi.fs_config(num_envs=4)), C.byref(h)), h.value)\n"
               "print(L.fs_last_error(None).decode())\n" % rocm[-1])
    images, rc, msg = out.strip().splitlines()[-3:]
    assert images.count("hsa:") == 2, images
    assert rc.split() == [str(_abi.FS_E_RUNTIME), "None"], rc
    assert "two HSA runtimes" in msg and os.path.realpath(rocm[-1]) in msg and "torch" in msg, msg


def test_library_loads_without_torch():
    """The C-ABI binding does not need torch (the reference client needs only gymnasium): with torch
    made unimportable, lib() loads the library on /opt/rocm's runtime, the host-only entry points
    answer, library_info reports the in-tree library, and fs_create without a device fails loudly."""
    out = _run("import sys; sys.modules['torch'] = None\n"
               "import ctypes as C\n"
               "from footsies_gym_amd import _lib, _abi\n"
               "L = _lib.lib()\n"
               "info = _lib.library_info()\n"
               "print(info['override'], info['path'], info['hip_build'] > 0)\n"
               "h = C.c_void_p()\n"
               "print(L.fs_create(C.byref(_abi.fs_config(num_envs=4)), C.byref(h)))\n"
               "print('torch' in sys.modules and sys.modules['torch'] is not None)\n")
    lines = out.strip().splitlines()[-3:]
    assert lines[0] == "False footsies_gym_amd/libfootsies.so True", lines
    assert int(lines[1]) in (_abi.FS_E_DEVICE, _abi.FS_OK), lines
    assert lines[2] == "False"


def test_library_override_is_reported(tmp_path):
    """FOOTSIES_LIB (kernel A/B experiments) swaps the library loudly: a note on stderr and
    library_info()['override'] (bench.py carries it in its line)."""
    import shutil
    import sys
    from footsies_gym_amd import build
    build.build()
    alt = tmp_path / "libfootsies.so"
    shutil.copy(build.LIB, alt)
    r = subprocess.run([sys.executable, "-c", "from footsies_gym_amd import _lib; print(_lib.library_info()['override'])"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=dict(os.environ, FOOTSIES_LIB=str(alt)))
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split()[-1] == "True"
    assert "FOOTSIES_LIB overrides" in r.stderr


def test_native_backend_without_device_fails_loudly():
    """FootsiesSim's torch-free backend: device outputs need torch (ImportError naming the way out);
    with host outputs and no device, fs_create's error surfaces as FootsiesError -- no CPU fallback."""
    out = _run("import sys; sys.modules['torch'] = None\n"
               "from footsies_gym_amd.simulator import FootsiesSim\n"
               "from footsies_gym_amd._lib import FootsiesError\n"
               "try:\n"
               "    FootsiesSim(8)\n"
               "except ImportError as e:\n"
               "    print('import-error', 'host_outputs=True' in str(e))\n"
               "try:\n"
               "    FootsiesSim(8, host_outputs=True)\n"
               "    print('created')\n"
               "except FootsiesError as e:\n"
               "    print('footsies-error', e.code)\n")
    lines = out.strip().splitlines()[-2:]
    assert lines[0] == "import-error True", lines
    assert lines[1] in ("footsies-error %d" % _abi.FS_E_DEVICE, "created"), lines
