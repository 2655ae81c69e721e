"""The -D USE_HIP shim (slam-indoor-code_amd/shim/*.cpp)
compiled and linked on the CPU.

The shim replaces the reference's OpenCV / Ceres call sites inside the
reference tree (CMakeLists.txt:56-67 picks one source set at compile time).
This image has no OpenCV, Ceres or reference build, so the shim is compiled
against tests/shim_stub/: stand-ins with OpenCV 4.8's names and layouts and the
reference's own signatures (featureMatching.h:12-53, fastExtractor.h:19-21,
bundleAdjustment.h:50-54, featureMatchingCommon.h:8-12), laid out so the shim's
relative includes ("../../config/config.h", "../../misc/IOmisc.h") resolve as
they would in src/mainModule/<module>/.  A caller that invokes every replaced
entry point through those declared signatures is then linked against the shim
objects and libslamhip_host / libslamhip: a signature or type that drifts from
the reference's fails to compile or leaves an undefined symbol.  Nothing runs
(no GPU here).  This is not a build of the reference.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-indoor-code_amd")
STUB = os.path.join(ROOT, "tests", "shim_stub")
SHIMS = {"featureMatchingHIP.cpp": "featureMatching", "fastExtractorHIP.cpp": "featureExtraction",
         "bundleAdjustmentHIP.cpp": "bundleAdjustment"}


def _gxx(args, cwd):
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror"] + args, cwd=cwd, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    return r


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    t = tmp_path_factory.mktemp("shimtree")
    shutil.copytree(os.path.join(STUB, "ref"), t / "ref")
    main = t / "ref" / "src" / "mainModule"
    for f, sub in SHIMS.items():
        os.makedirs(main / sub, exist_ok=True)
        shutil.copy(os.path.join(PKG, "shim", f), main / sub / f)
    shutil.copy(os.path.join(STUB, "caller.cpp"), main / "caller.cpp")
    return t


def _incs(tree):
    return ["-I", os.path.join(STUB), "-I", os.path.join(ROOT, "include"), "-I", os.path.join(PKG, "host"),
            "-I", str(tree / "ref" / "src" / "mainModule")]


@pytest.mark.parametrize("name", sorted(SHIMS))
def test_shim_compiles(tree, name):
    src = tree / "ref" / "src" / "mainModule" / SHIMS[name] / name
    _gxx(_incs(tree) + ["-c", str(src), "-o", str(src) + ".o"], cwd=str(src.parent))


def test_shim_links_with_reference_signatures(tree):
    if not os.path.exists(os.path.join(PKG, "slamhip", "libslamhip_host.so")):
        pytest.skip("libslamhip_host.so not built (make -C slam-indoor-code_amd)")
    main = tree / "ref" / "src" / "mainModule"
    objs = []
    for name, sub in SHIMS.items():
        src = main / sub / name
        _gxx(_incs(tree) + ["-c", str(src), "-o", str(src) + ".o"], cwd=str(src.parent))
        objs.append(str(src) + ".o")
    _gxx(_incs(tree) + ["-c", str(main / "caller.cpp"), "-o", str(main / "caller.o")], cwd=str(main))
    lib = os.path.join(PKG, "slamhip")
    rocm = "/opt/rocm/lib"
    _gxx([str(main / "caller.o")] + objs + ["-L", lib, "-lslamhip_host", "-lslamhip", "-L", rocm,
                                            f"-Wl,-rpath-link,{rocm}", "-o", str(main / "linked")], cwd=str(main))
    assert os.path.exists(main / "linked")
