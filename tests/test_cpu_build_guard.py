"""The shipped library's gfx950 code objects contain no packed fp32 VALU instructions (v_pk_fma_f32 /
v_pk_add_f32 / v_pk_mul_f32). csrc/Makefile builds the device code with NOPK (-packed-fp32-ops): their
low-half results came out wrong while other kernels of this library shared the CU.
This test makes that guard enforced rather than remembered: it unbundles every code object in the built
.so (objcopy + clang-offload-bundler, no GPU) and disassembles it."""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "rcnn-ocr_amd", "crnn_hip", "libcrnn_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
PACKED = re.compile(r"\bv_pk_(fma|add|mul)_f32\b")


def code_objects(tmp):
    fat = os.path.join(tmp, "fatbin")
    # objcopy with no output file rewrites its input in place: work on a copy (the shipped library may be
    # mapped by this very process, and an in-place rewrite under a mapping ends in SIGBUS)
    so = os.path.join(tmp, "lib.so")
    shutil.copyfile(SO, so)
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", so, os.path.join(tmp, "discard.so")],
                   check=True, capture_output=True)
    blob = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
    assert starts, "no offload bundle in .hip_fatbin"
    out = []
    for n, (a, b) in enumerate(zip(starts, starts[1:] + [len(blob)])):
        part = os.path.join(tmp, f"bundle{n}")
        with open(part, "wb") as f:
            f.write(blob[a:b])
        co = os.path.join(tmp, f"co{n}.o")
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={co}"],
                       check=True, capture_output=True)
        out.append(co)
    return out


def test_shipped_code_objects_have_no_packed_fp32(tmp_path):
    if not os.path.exists(SO):
        pytest.skip("libcrnn_hip.so not built")
    if not (shutil.which("objcopy") and os.path.exists(os.path.join(LLVM, "llvm-objdump"))):
        pytest.skip("objcopy / llvm-objdump not available")
    cos = code_objects(str(tmp_path))
    n_mfma, bad = 0, []
    for co in cos:
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co], check=True, capture_output=True,
                             text=True).stdout
        n_mfma += dis.count("v_mfma")
        bad += [l.strip() for l in dis.splitlines() if PACKED.search(l)][:5]
    assert n_mfma > 1000, f"{len(cos)} code objects, only {n_mfma} MFMAs: not the library's kernels?"
    assert not bad, f"packed fp32 instructions in the shipped gfx950 code: {bad}"
