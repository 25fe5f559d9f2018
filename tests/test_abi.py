"""C-ABI surface: libmipx.so loads on a CPU-only host and exports every symbol
include/mipx.h declares; the ctypes mirror matches the C struct layout."""
import ctypes
import os
import re
import subprocess

import numpy as np

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mipx.h")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mipx_\w+)\s*\(", text)))


def test_library_loads_and_exports_every_declared_symbol():
    import imaginary_amd as ia
    syms = header_symbols()
    assert len(syms) >= 40
    missing = [s for s in syms if not hasattr(ia.lib, s)]
    assert not missing, missing
    # the ctypes signature table covers the whole header too
    from imaginary_amd._abi import _SIG
    assert sorted(_SIG) == syms


def test_version_and_errors_without_gpu():
    import imaginary_amd as ia
    assert ia.lib.mipx_abi_version() == 6
    assert ia.lib.mipx_strerror(-9) == b"requests in flight"
    assert b"gfx950" in ia.lib.mipx_version()
    assert ia.lib.mipx_strerror(-2).startswith(b"operation not supported")


def test_struct_layout_matches_c(tmp_path):
    from imaginary_amd import _abi
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mipx.h"\n'
                   'int main(){printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(mipx_opts), '
                   'sizeof(mipx_input), sizeof(mipx_step), sizeof(mipx_plan), sizeof(mipx_img), '
                   'sizeof(mipx_cfg), offsetof(mipx_opts, sigma), offsetof(mipx_plan, steps));}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    C = ctypes
    want = [C.sizeof(_abi.MipxOpts), C.sizeof(_abi.MipxInput), C.sizeof(_abi.MipxStep),
            C.sizeof(_abi.MipxPlan), C.sizeof(_abi.MipxImg), C.sizeof(_abi.MipxCfg),
            _abi.MipxOpts.sigma.offset, _abi.MipxPlan.steps.offset]
    assert got == want


def test_init_without_device_reports_enodev():
    import imaginary_amd as ia
    if ia.device_count() > 0:
        pytest.skip("a device is visible")
    assert ia.lib.mipx_init(None) == -4


def test_product_does_not_import_oracle():
    """The oracle is a checker only: no product source may load or call it."""
    pkg = os.path.join(ROOT, "imaginary_amd")
    bad = re.compile(r"(import\s+oracle|from\s+oracle|liboracle|vips_ref\.h|\bref_[a-z]+\s*\()")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                assert not bad.search(open(os.path.join(dirpath, f)).read()), f
    out = subprocess.run(["nm", "-D", os.path.join(pkg, "libmipx.so")], capture_output=True, text=True).stdout
    assert "ref_" not in out and "liboracle" not in out


def test_entry_points_reject_bad_arguments_without_touching_the_device():
    """Every mipx_op_* validates its arguments before any HIP call: NULL pointers,
    empty or oversized batches and bad geometry return MIPX_EINVAL (-1)."""
    import imaginary_amd as ia
    L = ia.lib
    EINVAL = -1
    assert L.mipx_op_reduce(None, None, 1, 8, 8, 3, 2.0, 2.0, None, 0, None) == EINVAL
    assert L.mipx_op_reduce(1, 1, 0, 8, 8, 3, 2.0, 2.0, None, 0, None) == EINVAL
    assert L.mipx_op_reduce(1, 1, 1, 8, 8, 5, 2.0, 2.0, None, 0, None) == EINVAL
    assert L.mipx_op_reduce(1, 1, 1, 8, 8, 3, 0.5, 2.0, None, 0, None) == EINVAL
    assert L.mipx_op_shrink(1, 1, 1, 8, 8, 3, 0, 2, None) == EINVAL
    assert L.mipx_op_extract(1, 1, 1, 8, 8, 3, 4, 4, 8, 8, None) == EINVAL
    assert L.mipx_op_embed(1, 1, 1, 8, 8, 3, 0, 0, 0, 8, 1, None, None) == EINVAL
    assert L.mipx_op_affine(1, 1, 1, 8, 8, 3, 0.0, 2.0, 1, None) == EINVAL
    assert L.mipx_op_zoom(1, 1, 1, 8, 8, 3, 0, 2, None) == EINVAL
    assert L.mipx_op_watermark(1, 1, 1, 1, 8, 8, 3, 0, 4, 4, 0, 0, 1.0, None) == EINVAL
    assert L.mipx_op_gaussblur(None, 1, 1, 8, 8, 3, 2.0, 0.2, None, 0, None) == EINVAL
    assert L.mipx_op_flatten(None, 1, 1, 8, 8, 4, None, None) == EINVAL
    assert L.mipx_op_colourspace_bw(1, None, 1, 8, 8, 3, None) == EINVAL
    assert L.mipx_execute_dev(None, 1, 1, 1, None, None, 0, None) == EINVAL


def test_request_api_before_init():
    import ctypes as C
    import imaginary_amd as ia
    t = C.c_uint64()
    assert ia.lib.mipx_wait(12345, 0) == -8           # unknown ticket
    assert ia.lib.mipx_stats(0, C.byref(t), C.byref(t)) in (-7, -1, 0)


def _ashr_pk_feeds(dis: str):
    """For every v_ashr_pk_u8_i32 in a disassembly, the mnemonic of the first later
    instruction that reads its destination (None when it is overwritten or unused)."""
    import re
    lines = [l.split(";")[0].strip() for l in dis.splitlines()]
    lines = [l for l in lines if re.match(r"^[sv]_|^ds_|^buffer_|^global_", l)]
    out = []
    for i, l in enumerate(lines):
        if not l.startswith("v_ashr_pk_u8_i32"):
            continue
        dst = l.split()[1].rstrip(",")
        use = None
        for m in lines[i + 1:i + 200]:
            parts = m.replace(",", " ").split()
            if dst in parts[2:]:
                use = parts[0]
                break
            if len(parts) > 1 and parts[1] == dst:
                break
        out.append(use)
    return out


def test_code_object_avoids_known_bad_gfx950_fusion(tmp_path):
    """The gfx950 backend can fuse shift + clamp + byte packing into
    v_ashr_pk_u8_i32 and then OR the next channels into its unwritten upper half
    as if it were zero (a channel-2 error found by the whole-plan fuzz).
    fixed_round_i keeps the backend from fusing; round_pack4 uses the instruction
    on purpose and joins the two 16-bit halves with v_perm_b32.  So every
    v_ashr_pk_u8_i32 in the shipped code must feed a v_perm_b32, never an OR."""
    import shutil
    import imaginary_amd as ia
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not available")
    so = tmp_path / "libmipx.so"
    shutil.copy(ia.LIB_PATH, so)
    subprocess.run([objdump, "--offloading", str(so)], cwd=tmp_path, check=True, capture_output=True)
    objs = [p for p in tmp_path.iterdir() if "gfx950" in p.name]
    assert objs, "no gfx950 code object in libmipx.so"
    seen_dot2 = False
    for p in objs:
        dis = subprocess.run([objdump, "-d", "--mcpu=gfx950", str(p)], check=True, capture_output=True, text=True).stdout
        seen_dot2 |= "v_dot2_i32_i16" in dis or "v_dot2c_i32_i16" in dis
        feeds = _ashr_pk_feeds(dis)
        bad = [f for f in feeds if f not in ("v_perm_b32", None)]
        assert not bad, f"{p.name}: v_ashr_pk_u8_i32 feeding {sorted(set(bad))}"
    assert seen_dot2, "disassembly lacks the reduce passes' dot2 (extraction failed?)"


def test_shipped_library_carries_no_unreachable_kernels_or_probes(tmp_path):
    """kernels no default dispatch reaches (r05's k_rchain,
    k_reduce2d, k_reduce2w and the k_enlm-shadowed k_enlarge2) are gone from the
    product library (their A/B records stay under profiles/), and the pixel-corrupting
    timing probes (MIPX_ENLM_DBG) and the launch-geometry dump (MIPX_BCOL_DBG) exist
    only in a `make PROBES=1` build (libmipx_probes.so), never in libmipx.so."""
    import shutil
    import imaginary_amd as ia
    syms = subprocess.run(["nm", "-C", ia.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "k_reduce2x2<3, 66>" in syms and "k_enlm<" in syms   # the listing does name kernels
    for k in ("k_rchain", "k_reduce2d", "k_reduce2w", "k_enlarge2"):
        assert k not in syms, k
    with open(ia.LIB_PATH, "rb") as f:
        blob = f.read()
    for knob in (b"MIPX_ENLM_DBG", b"MIPX_BCOL_DBG", b"MIPX_CHAIN", b"MIPX_R2D", b"MIPX_R2_WALK", b"MIPX_ENLARGE2"):
        assert knob not in blob, knob
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if os.path.exists(objdump):  # nor in the device code objects
        so = tmp_path / "libmipx.so"
        shutil.copy(ia.LIB_PATH, so)
        subprocess.run([objdump, "--offloading", str(so)], cwd=tmp_path, check=True, capture_output=True)
        kern = "".join(subprocess.run(["nm", "-C", str(p)], capture_output=True, text=True).stdout
                       for p in tmp_path.iterdir() if "gfx950" in p.name)
        assert "k_enlm" in kern and "k_reduce2m" in kern
        assert not any(k in kern for k in ("k_rchain", "k_reduce2d", "k_reduce2w", "k_enlarge2"))


def test_build_id_is_the_hash_of_these_sources():
    """Build provenance: libmipx.so carries the hash of the sources it was built
    from (imaginary_amd/srchash.py); it must be the hash of this tree's sources."""
    import imaginary_amd as ia
    from imaginary_amd.srchash import source_hash
    assert ia.lib.mipx_build_id().decode() == source_hash()
    assert ia.lib.mipx_build_id() in ia.lib.mipx_version()


def build_c_client(dst):
    """gcc-compile tests/c/mipx_client.c against include/mipx.h (plain C, as the cgo
    shim would), linked to libmipx.so and the oracle (checker)."""
    from oracle import oracle as o
    o.build()
    exe = os.path.join(str(dst), "mipx_client")
    subprocess.run(["gcc", "-O2", "-Wall", "-Wextra", "-Werror", "-std=c11", "-D_DEFAULT_SOURCE",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "tests", "c", "mipx_client.c"),
                    "-L", os.path.join(ROOT, "imaginary_amd"), "-L", os.path.join(ROOT, "oracle", "_build"),
                    "-lmipx", "-loracle", "-lpthread",
                    "-Wl,-rpath," + os.path.join(ROOT, "imaginary_amd") + ":" + os.path.join(ROOT, "oracle", "_build"),
                    "-o", exe], check=True)
    return exe


def build_c_e2e(dst):
    """gcc-compile tests/c/mipx_e2e.c (the request-path throughput benchmark from C)."""
    exe = os.path.join(str(dst), "mipx_e2e")
    subprocess.run(["gcc", "-O2", "-Wall", "-Wextra", "-Werror", "-std=c11", "-D_DEFAULT_SOURCE",
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "c", "mipx_e2e.c"),
                    "-L", os.path.join(ROOT, "imaginary_amd"), "-lmipx", "-lpthread",
                    "-Wl,-rpath," + os.path.join(ROOT, "imaginary_amd"), "-o", exe], check=True)
    return exe


def test_c_e2e_builds_against_the_header(tmp_path):
    assert os.path.exists(build_c_e2e(tmp_path))


def test_c_client_builds_against_the_header(tmp_path):
    exe = build_c_client(tmp_path)
    import imaginary_amd as ia
    if ia.device_count() == 0:
        r = subprocess.run([exe], capture_output=True, text=True)
        assert r.returncode == 77, r.stderr


def _plan_reduce_2x(ia):
    return ia.plan_make(ia.make_opts(width=160, height=120, embed=1), ia.make_input(320, 240, 3, "png"))


def test_inconsistent_plans_are_rejected_before_any_device_work():
    """plans are ABI data; a step whose stated geometry disagrees with
    its op must be EINVAL at mipx_workspace_bytes / mipx_execute_dev / mipx_submit,
    never a kernel writing past a buffer sized for the stated geometry."""
    import ctypes as C
    import imaginary_amd as ia
    from imaginary_amd import _abi
    L = ia.lib
    good = _plan_reduce_2x(ia)
    cases = []
    p = _abi.MipxPlan.from_buffer_copy(good)          # reduce says 170 wide, makes 160
    p.steps[0].out_w = 170
    p.out_w = 170
    cases.append(p)
    p = _abi.MipxPlan.from_buffer_copy(good)          # embed step grows past the stated size
    p.n_steps = 2
    s = p.steps[1]
    s.op = _abi.OP_EMBED
    s.a[2], s.a[3], s.a[4] = 400, 300, 1
    s.out_w, s.out_h, s.out_bands = 160, 120, 3
    cases.append(p)
    p = _abi.MipxPlan.from_buffer_copy(good)          # zoom writes w*xf x h*yf
    p.n_steps = 1
    p.steps[0].op = _abi.OP_ZOOM
    p.steps[0].a[0] = p.steps[0].a[1] = 2
    p.steps[0].out_w, p.steps[0].out_h = 160, 120
    cases.append(p)
    p = _abi.MipxPlan.from_buffer_copy(good)          # smartcrop larger than its input
    p.n_steps = 1
    p.steps[0].op = _abi.OP_SMARTCROP
    p.steps[0].a[0], p.steps[0].a[1] = 400, 100
    p.steps[0].out_w, p.steps[0].out_h = p.out_w, p.out_h = 400, 100
    cases.append(p)
    p = _abi.MipxPlan.from_buffer_copy(good)          # reduce with no such sampling convention
    p.steps[0].a[7] = 2
    cases.append(p)
    p = _abi.MipxPlan.from_buffer_copy(good)          # extract outside the image
    p.n_steps = 1
    p.steps[0].op = _abi.OP_EXTRACT
    p.steps[0].a[:4] = [300, 0, 40, 40]
    p.steps[0].out_w, p.steps[0].out_h = p.out_w, p.out_h = 40, 40
    cases.append(p)
    for bad in cases:
        assert L.mipx_workspace_bytes(C.byref(bad), 1) == 0
        assert L.mipx_execute_dev(C.byref(bad), 1, 16, 16, None, 16, 1 << 30, None) == -1
        src = np.zeros((bad.in_h, bad.in_w, bad.in_bands), np.uint8)
        dst = np.zeros((bad.out_h, bad.out_w, bad.out_bands), np.uint8)
        t = C.c_uint64()
        assert L.mipx_submit(-1, C.byref(bad), C.byref(_img(src)), None, C.byref(_img(dst)), C.byref(t)) == -1


def _img(a):
    from imaginary_amd._abi import MipxImg
    return MipxImg(a.ctypes.data, a.shape[1], a.shape[0], a.shape[2], a.strides[0])


def test_watermark_image_must_match_the_plan():
    """the watermark kernel reads with the step's wm geometry, so a
    caller's watermark of another size is EINVAL at submit."""
    import ctypes as C
    import imaginary_amd as ia
    L = ia.lib
    p = ia.plan_make(ia.make_opts(width=256, height=192, wm_enable=1, wm_left=16, wm_top=16, wm_opacity=0.5),
                     ia.make_input(400, 300, 3, "png", 0, wm_w=128, wm_h=128, wm_bands=4))
    src = np.zeros((300, 400, 3), np.uint8)
    dst = np.zeros((p.out_h, p.out_w, p.out_bands), np.uint8)
    t = C.c_uint64()
    for shape in [(64, 64, 4), (128, 128, 3), (128, 127, 4)]:
        wm = np.zeros(shape, np.uint8)
        assert L.mipx_submit(-1, C.byref(p), C.byref(_img(src)), C.byref(_img(wm)), C.byref(_img(dst)),
                             C.byref(t)) == -1
    assert L.mipx_submit(-1, C.byref(p), C.byref(_img(src)), None, C.byref(_img(dst)), C.byref(t)) == -1


def test_plan_records_the_sampling_convention():
    """ABI v6: mipx_plan_make stores the process's reduce sampling
    convention in every REDUCE / SMARTCROP step (a[7]); flipping the setting later does
    not change a plan already made, and the setter works with nothing in flight."""
    import imaginary_amd as ia
    prev = ia.reduce_sampling()
    try:
        ia.set_reduce_sampling("corner")
        corner = _plan_reduce_2x(ia)
        smart_c = ia.plan_make(ia.make_opts(width=64, height=64, crop=1, gravity=5), ia.make_input(320, 240, 3, "png"))
        ia.set_reduce_sampling("centre")
        centre = _plan_reduce_2x(ia)
        smart_m = ia.plan_make(ia.make_opts(width=64, height=64, crop=1, gravity=5), ia.make_input(320, 240, 3, "png"))
        assert corner.steps[0].a[7] == 0 and centre.steps[0].a[7] == 1
        assert [s[0] for s in smart_m.describe()][-1] == "smartcrop"
        assert smart_c.steps[smart_c.n_steps - 1].a[7] == 0 and smart_m.steps[smart_m.n_steps - 1].a[7] == 1
        assert corner.steps[0].a[7] == 0                      # the earlier plan kept its convention
        assert ia.lib.mipx_set_reduce_sampling(5) == -1
    finally:
        ia.set_reduce_sampling(prev)
