"""The C-ABI library builds for gfx950, loads, and exports every symbol include/admm_tv.h declares.

Host-only entry points (version, size checks, workspace sizing, error codes) are
exercised; nothing here launches a kernel (no GPU in the build container).
"""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "admm_tv.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(admm_tv_\w+)\s*\(", txt)))


def test_header_and_binding_agree():
    from admmtor import _native
    assert declared_functions() == sorted(_native.EXPORTED)


def test_library_exports_every_declared_symbol():
    from admmtor import _native
    so = _native.lib_path()
    assert os.path.exists(so), "build the library first (python __graft_entry__.py build)"
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s(admm_tv_\w+)", out))
    missing = set(declared_functions()) - exported
    assert not missing, missing
    lib = _native.load()
    for name in declared_functions():
        assert getattr(lib, name) is not None


def test_library_is_gfx950_code():
    from admmtor import _native
    blob = open(_native.lib_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the embedded code object targets gfx950 only
    assert b"gfx942" not in blob and b"sm_" not in blob[:0]  # no other GPU target bundled


def test_host_entry_points():
    from admmtor import _native
    lib = _native.load()
    assert lib.admm_tv_abi_version() == 7
    fast, generic = 1, 2
    assert [lib.admm_tv_supported(*hw) for hw in ((1024, 1024), (16, 2048), (4096, 16))] == [fast] * 3
    assert [lib.admm_tv_supported(*hw) for hw in ((15, 17), (1024, 8192), (8, 64), (1, 1), (509, 321))] == [generic] * 5
    assert [lib.admm_tv_supported(*hw) for hw in ((321, 481), (481, 321))] == [4] * 2  # odd-length rows, either way
    assert [lib.admm_tv_supported(*hw) for hw in ((4097, 16), (5000, 33))] == [generic] * 2  # beyond 4096
    assert [lib.admm_tv_supported(*hw) for hw in ((65537, 16), (16, 70000), (0, 16))] == [0] * 3
    # smooth sizes with transform plans: the fused iteration on mixed-radix transforms (inference)
    assert [lib.admm_tv_supported(*hw) for hw in ((1080, 1920), (720, 1280), (480, 640), (2160, 512), (2160, 3840),
                                                  (1024, 4096), (4096, 4096), (600, 800), (1200, 1600), (1440, 2560),
                                                  (1536, 2048))] == [3] * 11
    assert [lib.admm_tv_supported(*hw) for hw in ((1080, 7680), (1081, 1920), (1080, 1918))] == [generic] * 3
    d = _native.desc(64, 3, 1024, 1024, 21, False, 50)
    ws = _native.workspace_size(d)
    img = 64 * 3 * 1024 * 1024 * 4
    assert 7 * img <= ws <= 7 * img + (64 << 20)  # 2 spectra + 4 u + b (+ small tables)
    d_iso = _native.desc(16, 3, 512, 512, 0, True, 100)
    assert _native.workspace_size(d_iso) > 6 * 16 * 3 * 512 * 512 * 4


def test_host_entry_points_f64():
    """fp64 solves (ADMM_TV_FLAG_F64): every size the double kernels' LDS image admits, fp64 sizes,
    and the precision of a descriptor and of an entry point must agree."""
    from admmtor import _native
    lib = _native.load()
    assert [lib.admm_tv_supported_f64(*hw) for hw in ((1024, 1024), (15, 17), (1, 1), (481, 321), (256, 4096))] \
        == [1] * 5
    assert [lib.admm_tv_supported_f64(*hw) for hw in ((65537, 16), (0, 16))] == [0] * 2
    assert lib.admm_tv_supported_f64(6000, 12000) == 1  # fp64 lines beyond 5,120 points: global buffers
    d32 = _native.desc(2, 3, 64, 96, 5, False, 10)
    d64 = _native.desc(2, 3, 64, 96, 5, False, 10, f64=True)
    assert d64.flags & _native.ADMM_TV_FLAG_F64
    img = 2 * 3 * 64 * 96
    assert _native.workspace_size(d64) >= 7 * img * 8 > _native.workspace_size(d32)
    assert _native.history_size(_native.desc(2, 3, 64, 96, 5, False, 10, f64=True)) == \
        2 * _native.history_size(_native.desc(2, 3, 64, 96, 5, False, 10))
    # an fp32 entry point refuses an fp64 descriptor (and vice versa) before touching any pointer
    assert lib.admm_tv_forward(ctypes.byref(d64), None, None, None, None, None, None, 0, None) == _native.ADMM_TV_EINVAL
    assert lib.admm_tv_forward_f64(ctypes.byref(d32), None, None, None, None, None, None, 0, None) == \
        _native.ADMM_TV_EINVAL
    assert b"f64" in lib.admm_tv_last_error()
    dg = _native.desc(2, 3, 64, 64, 0, False, 10, groups=2, f64=True)
    n = ctypes.c_size_t(0)
    assert lib.admm_tv_workspace_size(ctypes.byref(dg), ctypes.byref(n)) == _native.ADMM_TV_EUNSUPPORTED


@pytest.mark.parametrize("field,value,code", [
    ("kw", 5, -3),      # non-square PSF -> ADMM_TV_ENONSQUARE
    ("H", 65537, -2),   # unsupported size (a line longer than 65,536 points)
    ("maxit", -1, -1),  # invalid
    ("kh", 99, -3),
])
def test_host_error_codes(field, value, code):
    from admmtor import _native
    d = _native.desc(1, 1, 64, 64, 3, False, 5)
    setattr(d, field, value)
    n = ctypes.c_size_t(0)
    assert _native.load().admm_tv_workspace_size(ctypes.byref(d), ctypes.byref(n)) == code
    assert _native.load().admm_tv_last_error()


def test_empty_shard_needs_an_iso_hook():
    """B*C = 0 is invalid for a plain solve, valid for an iso solve with a cross-rank hook (an empty
    shard still takes part in every all-reduce; ABI v4 carries the hook in the descriptor)."""
    from admmtor import _native
    lib = _native.load()
    n = ctypes.c_size_t(0)
    d = _native.desc(0, 3, 64, 64, 0, True, 5)
    assert lib.admm_tv_workspace_size(ctypes.byref(d), ctypes.byref(n)) == -1
    d.allreduce = _native.ALLREDUCE_FN(lambda *a: None)
    assert lib.admm_tv_workspace_size(ctypes.byref(d), ctypes.byref(n)) == 0 and n.value >= 2 * 64 * 64 * 4
    d.iso = 0  # the hook is only for iso
    assert lib.admm_tv_workspace_size(ctypes.byref(d), ctypes.byref(n)) == -1


def test_psf_larger_than_image_is_rejected():
    from admmtor import _native
    d = _native.desc(1, 1, 16, 16, 21, False, 5)
    n = ctypes.c_size_t(0)
    assert _native.load().admm_tv_workspace_size(ctypes.byref(d), ctypes.byref(n)) == -6


def test_groups_descriptor():
    """desc.groups = G: G modules sharing xin -> G x the per-plane state, G Wiener factors."""
    from admmtor import _native
    one = _native.workspace_size(_native.desc(16, 3, 512, 512, 0, True, 100))
    two = _native.workspace_size(_native.desc(16, 3, 512, 512, 0, True, 100, 0, 2))
    # per-module state doubles; b (one image, shared by the modules) and the tables do not
    img = 16 * 3 * 512 * 512 * 4
    assert 1.7 * one < two < 2.1 * one and two - one > 6 * img
    h1 = _native.history_size(_native.desc(16, 3, 512, 512, 0, True, 10))
    h2 = _native.history_size(_native.desc(16, 3, 512, 512, 0, True, 10, 0, 2))
    assert abs(h2 - 2 * h1) < (1 << 16)
    n = ctypes.c_size_t(0)
    lib = _native.load()
    # generic sizes and PSF gradients are not grouped
    assert lib.admm_tv_workspace_size(ctypes.byref(_native.desc(1, 1, 15, 17, 0, False, 5, 0, 2)), ctypes.byref(n)) == -2
    assert lib.admm_tv_workspace_size(ctypes.byref(_native.desc(1, 1, 64, 64, 3, False, 5, 1, 2)), ctypes.byref(n)) == -2
    assert lib.admm_tv_workspace_size(ctypes.byref(_native.desc(1, 1, 64, 64, 0, False, 5, 0, -1)), ctypes.byref(n)) == -1


def test_library_built_from_this_tree():
    """admm_tv_build_hash() (embedded by csrc/Makefile) equals the hash of the sources in the tree,
    so a stale prebuilt library cannot pass for the current code (load() refuses it too)."""
    from admmtor import _native
    assert _native.load().admm_tv_build_hash().decode() == _native.source_hash()


def test_supported_sizes():
    """admm_tv_supported (host-only): power-of-two sizes on the fused kernels (1), any other size up
    to 65,536 per side on the generic kernels (2; twiddles move to global memory beyond ~6,800
    points, the line buffers too beyond 10,240), else 0."""
    from admmtor import _native
    L = _native.load()
    assert L.admm_tv_supported(1024, 1024) == 1 and L.admm_tv_supported(4096, 2048) == 1
    assert L.admm_tv_supported(15, 17) == 2 and L.admm_tv_supported(4096, 4096) == 3
    assert L.admm_tv_supported(6000, 4000) == 2 and L.admm_tv_supported(6800, 16) == 2
    assert L.admm_tv_supported(7680, 4320) == 2 and L.admm_tv_supported(8192, 8192) == 2  # global twiddles
    assert L.admm_tv_supported(10240, 16) == 2 and L.admm_tv_supported(10241, 16) == 2  # global line buffers
    assert L.admm_tv_supported(1, 12000) == 2 and L.admm_tv_supported(65536, 3) == 2
    assert L.admm_tv_supported(65537, 16) == 0 and L.admm_tv_supported(0, 16) == 0
    # long lines' scratch slots are part of the workspace, bounded by the items of one launch
    from admmtor import _native as nat
    small = nat.workspace_size(nat.desc(1, 1, 1, 12000, 0, False, 5))
    assert small < (16 << 20)  # one 12,000-point row: one slot, not 1,024
    big = nat.workspace_size(nat.desc(2, 3, 12000, 12000, 0, False, 5))
    assert big >= 7 * 2 * 3 * 12000 * 12000 * 4


# ---------------------------------------------------------------- frozen release library
CSRC = os.path.join(ROOT, "torch-admm-deconv_amd", "csrc")
RUNTIME_SETTINGS = {"ADMM_GEN_STREAMS"}  # documented in INTEGRATION.md (and csrc/knobs.hpp)


def _sources():
    for name in sorted(os.listdir(CSRC)):
        if name.endswith((".hip", ".hpp")):
            yield name, open(os.path.join(CSRC, name)).read()


def test_environment_reads_are_gated():
    """Every environment read of the library goes through knobs.hpp: getenv nowhere else; the
    env_setting names (read in every build) are exactly the documented runtime settings; every other
    name is an env_int A/B knob, which a release build (no -DADMM_AB_BUILD) compiles to its default."""
    settings, knobs = set(), set()
    for name, txt in _sources():
        code = re.sub(r"//[^\n]*", "", txt)
        if name != "knobs.hpp":
            assert "getenv" not in code, f"{name}: environment read outside knobs.hpp"
            assert "secure_getenv" not in code and "environ" not in code.replace("environment", ""), name
        settings |= set(re.findall(r'env_setting\(\s*"(ADMM_\w+)"', code))
        knobs |= set(re.findall(r'env_int\(\s*"?(ADMM_\w+|knob)', code))
    assert settings == RUNTIME_SETTINGS, settings
    knobs_hpp = open(os.path.join(CSRC, "knobs.hpp")).read()
    assert re.search(r"inline int env_int\(const char\* name, int dflt\) \{ return ADMM_AB_BUILD \?", knobs_hpp)
    assert re.search(r"#ifndef ADMM_AB_BUILD\s*#define ADMM_AB_BUILD 0", knobs_hpp)
    mk = open(os.path.join(CSRC, "Makefile")).read()
    # the release library's flags never turn the knobs on; only the separate A/B target does
    rules = "\n".join(ln for ln in mk.splitlines() if not ln.lstrip().startswith("#"))
    assert re.search(r"^EXTRA\s*\?=\s*$", mk, re.M) and rules.count("ADMM_AB_BUILD=1") == 1
    assert re.search(r"^ab:\n\t\$\(MAKE\) OBJDIR=build_ab OUT=\$\(AB_OUT\) EXTRA=-DADMM_AB_BUILD=1", mk, re.M)
    assert all(s in knobs_hpp for s in RUNTIME_SETTINGS)
    integ = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert all(s in integ for s in RUNTIME_SETTINGS)


# environment variables the Python package itself may read (admmtor/**/*.py), each documented in
# opt-outs to PyTorch's own statistics ops and the double backward's checkpoint
# segment length.  The library path is not among them: tools and tests pick an A/B variant through
# _native.use_library(), never the package through the environment.
PACKAGE_ENV = {"ADMMTOR_CHANPOOL", "ADMMTOR_PLANESTAT", "ADMM_SO_SEGMENT", "ADMM_SO_UNROLLED"}


def test_package_environment_reads_are_allowlisted():
    """Every os.environ / os.getenv read in the package names an allowlisted variable; no other access to
    the environment (a whole-environment scan, a computed name) exists."""
    found = set()
    for dirpath, _, files in os.walk(os.path.join(ROOT, "torch-admm-deconv_amd", "admmtor")):
        for fn in files:
            if not fn.endswith(".py"):
                continue
            path = os.path.join(dirpath, fn)
            code = re.sub(r"#[^\n]*", "", open(path).read())
            for m in re.finditer(r"os\.(environ|getenv)", code):
                tail = code[m.end():m.end() + 80]
                name = re.match(r'(?:\.get\(|\[|\()\s*"(\w+)"', tail)
                assert name, f"{fn}: environment access without a literal name: {tail[:40]!r}"
                found.add(name.group(1))
    assert found <= PACKAGE_ENV, found - PACKAGE_ENV
    integ = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert all(v in integ for v in found), [v for v in found if v not in integ]
    assert "ADMMTOR_LIB_OVERRIDE" not in open(os.path.join(ROOT, "torch-admm-deconv_amd", "admmtor",
                                                            "_native.py")).read()


def test_release_load_path_ignores_the_override(monkeypatch):
    """Setting ADMMTOR_LIB_OVERRIDE changes nothing for the package: a fresh interpreter loads the release
    library."""
    import subprocess
    import sys
    code = ("import sys; sys.path[:0] = [%r]\n"
            "from admmtor import _native\n"
            "_native.load()\n"
            "print(_native.lib_path())\n") % os.path.join(ROOT, "torch-admm-deconv_amd")
    env = dict(os.environ, ADMMTOR_LIB_OVERRIDE=os.path.join(CSRC, "..", "admmtor", "_lib", "libadmm_tv_ab.so"))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout.strip().endswith(os.path.join("_lib", "libadmm_tv.so"))


def test_release_library_ignores_ab_knobs():
    """The workspace layout depends on A/B knobs (the spectrum pitch, the mixed-radix path, the iso
    plane groups): in the release library, setting them changes nothing."""
    import sys
    code = ("import sys; sys.path[:0] = [%r]\n"
            "from admmtor import _native\n"
            "for hw in ((321, 481), (1080, 1920), (512, 512)):\n"
            "    for iso in (0, 1):\n"
            "        d = _native.AdmmTvDesc(B=4, C=3, H=hw[0], W=hw[1], kh=9, kw=9, iso=iso, maxit=5)\n"
            "        print(_native.workspace_size(d))\n") % os.path.join(ROOT, "torch-admm-deconv_amd")
    env0 = {k: v for k, v in os.environ.items() if not k.startswith("ADMM_")}
    env1 = dict(env0, ADMM_GEN_PITCH="0", ADMM_MIXED="0", ADMM_ISO_PPG="1", ADMM_GCOL_MM="0", ADMM_GROW_MM="0")
    outs = [subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, check=True).stdout
            for e in (env0, env1)]
    assert outs[0] == outs[1] and len(outs[0].split()) == 6
    # ... while the A/B build (admmtor._native.ab_library: tests comparing kernel paths) follows them
    code_ab = code.replace("from admmtor import _native\n", "from admmtor import _native\n_native._lib = _native._open(_native.AB_LIB_PATH)\n")
    ab = [subprocess.run([sys.executable, "-c", code_ab], env=e, capture_output=True, text=True, check=True).stdout
          for e in (env0, env1)]
    assert ab[0] == outs[0] and ab[1] != ab[0]
