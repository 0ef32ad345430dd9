"""The C-ABI boundary without a GPU: the library loads, exports every symbol the header
declares, and its host-side entries behave (errors, camera, PPM writer)."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
import raytracert_amd as R
from raytracert_amd import _capi
from _util import survey_pins, read_ppm


def test_library_exports_every_header_symbol():
    lib = _capi.lib()
    syms = _capi.header_symbols()
    assert len(syms) >= 17
    for s in syms:
        assert hasattr(lib, s), s
    # the Python binding declares a signature for every exported entry
    assert set(syms) == set(_capi._SIGNATURES)


def test_struct_layouts_match_header():
    # 8 int fields, 16 inline lights, camera, 8 corners, then the light_list pointer (8-aligned)
    assert C.sizeof(_capi.RtParams) == 4 * 8 + 16 * 12 + 12 + 8 * 12 + 4 + 8
    assert _capi.RtParams.light_list.offset == 336
    assert C.sizeof(_capi.RtMaterial) == 4 * 14
    assert C.sizeof(_capi.RtParams) == C.sizeof(O.OraParams)


def test_default_corners_bitwise_equal_oracle_and_pins():
    for w, h in [(64, 64), (800, 600), (1920, 1080), (3840, 2160), (48, 27)]:
        a = R.default_corners(w, h)
        b = O.default_corners(w, h)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    pins = survey_pins()["corners_1920x1080"]
    c = R.default_corners(1920, 1080)
    np.testing.assert_allclose(c[0], pins["o00"], atol=5e-7, rtol=0)
    np.testing.assert_allclose(c[7], pins["d11"], atol=5e-7, rtol=0)


def test_write_ppm_roundtrip(tmp_path):
    img = (np.arange(5 * 7 * 3) % 256).astype(np.uint8).reshape(5, 7, 3)
    p = str(tmp_path / "x.ppm")
    R.write_ppm(p, img)
    assert open(p, "rb").read(11) == b"P6\n7 5\n255\n"
    assert np.array_equal(read_ppm(p), img)


@pytest.mark.parametrize("threads", [1, 3, 16])
def test_ppm_writer_same_file(tmp_path, threads):
    """rt_ppm_writer_* (a mapped result.ppm written after every frame) leaves rt_write_ppm's file byte
    for byte, frame after frame, also over a larger previous file (sized at open)."""
    rng = np.random.default_rng(threads)
    a, b = str(tmp_path / "a.ppm"), str(tmp_path / "b.ppm")
    with open(b, "wb") as f:
        f.write(b"x" * (480 * 270 * 3 + 5000))
    with R.PpmWriter(b, 480, 270, threads) as w:
        for _ in range(3):
            img = rng.integers(0, 256, (270, 480, 3), dtype=np.uint8)
            w.write(img)
            R.write_ppm(a, img)
            assert open(a, "rb").read() == open(b, "rb").read()
        with pytest.raises(ValueError):
            w.write(img[:100])
    with pytest.raises(R.RtError):
        R.PpmWriter(b, 480, 270, 0)


def test_errors_are_codes_with_messages(tmp_path):
    with pytest.raises(R.RtError) as ei:
        R.default_corners(0, 10)
    assert ei.value.code == _capi.RT_E_ARG
    with pytest.raises(R.RtError) as ei:
        R.write_ppm(str(tmp_path / "nodir" / "x.ppm"), np.zeros((2, 2, 3), np.uint8))
    assert ei.value.code == _capi.RT_E_IO


def test_host_only_scene_refuses_render(tmp_path):
    p = tmp_path / "t.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    s = R.Scene.load(str(p), device=R.RT_HOST_ONLY)
    with pytest.raises(R.RtError) as ei:
        s.render(R.RenderParams(width=4, height=4, pf=1, max_lvl=0))
    assert ei.value.code == _capi.RT_E_NODEV
    with pytest.raises(R.RtError):
        s.intersect_mesh([[0, 0, 1]], [[0, 0, -1]])
    assert s.get_material(0)["Kd"] == (0.5, 0.5, 0.5)   # default material (mesh.cpp:108-117)


def test_scene_create_validates_indices():
    with pytest.raises(R.RtError) as ei:
        R.Scene.create([[0, 0, 0]], [[0, 0, 1]], [0], [dict(Kd=(1, 1, 1), flags=1)], device=R.RT_HOST_ONLY)
    assert ei.value.code == _capi.RT_E_PARSE
    s = R.Scene.create([[0, 0, 0], [1, 0, 0], [0, 1, 0]], [[0, 1, 2]], [0], [dict(Kd=(1, 1, 1), flags=1)],
                       device=R.RT_HOST_ONLY)
    assert s.counts() == (3, 1, 1)
    assert s.export()["normals"].tolist() == [[0.0, 0.0, 1.0]]


def test_comm_id_without_gpu_and_init_refusal():
    """rt_comm_unique_id loads RCCL on first use and makes fresh 128-byte ids; rt_comm_init
    checks its arguments before any collective (and needs a device)."""
    a, b = R.Comm.unique_id(), R.Comm.unique_id()
    assert len(a) == len(b) == _capi.COMM_ID_BYTES and a != b
    with pytest.raises(R.RtError) as ei:
        R.Comm(0, 1, 1, a)   # rank outside [0, nranks)
    assert ei.value.code == _capi.RT_E_ARG
    if R.device_count() == 0:
        with pytest.raises(R.RtError) as ei:
            R.Comm(0, 0, 1, a)
        assert ei.value.code == _capi.RT_E_NODEV


def test_tune_knobs_validate_ranges(tmp_path):
    """rt_scene_tune range checks on a host-only scene (no GPU): the launch-shape knobs accept
    their documented values and refuse others with RT_E_ARG; the knobs retired in r03 (measured
    slower, their kernels removed) accept only 0."""
    p = tmp_path / "t.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    s = R.Scene.load(str(p), device=R.RT_HOST_ONLY)
    for knob, good, bad in [("wave_steal", (0, 1, 2), (-1, 3)), ("chain_refill", (0,), (1,)),
                            ("refill_grid", (0,), (1, 2560)), ("wave_traversal", (0,), (1, -1)),
                            ("batch_order", (0, 1), (2, 3)), ("chain_split", (0, 3, 4, 5), (6, 7, -1)),
                            ("pixel_order", (0, 1, 2), (3, -1)), ("dyn_group", (0, 2, 6), (7, -1)),
                            ("cold_estimate", (0, 1, 2), (3, -1)),
                            ("steal_half", (0, 512, 65535), (-1, 65536)), ("steal_quarter", (-1, 0, 8, 4096), (-2, 4097)),
                            ("split_eighth", (0, 64, 4096), (-1, 4097)), ("prio_batches", (0, 64, 1 << 30), (-1,)),
                            ("shadow_helpers", (0, 1, 2), (3, -1)), ("quad_walk", (0, 1), (2, -1)), ("motion_order", (0, 1, 2, 8), (9, -1)), ("order_early", (0, 1), (2, -1)), ("frames_in_flight", (1, 2, 4), (0, 5)), ("pipes", (1, 4), (0, 5))]:
        for v in good:
            s.tune(knob, v)
        for v in bad:
            with pytest.raises(R.RtError):
                s.tune(knob, v)


def _layout(cap, steps, lights):
    total = C.c_uint64()
    ext = (C.c_uint64 * (2 * _capi.RT_WS_ARRAYS))()
    _capi.check(_capi.lib().rt_workspace_layout(cap, steps, lights, C.byref(total), ext))
    return int(total.value), np.array(ext, dtype=np.uint64).reshape(-1, 2)


@pytest.mark.parametrize("cap", [0, 1, 63, 64, 65, 1000, 4095, 2_073_600, 8_294_400 * 4])
@pytest.mark.parametrize("steps", [1, 2, 4, 11, 255])
@pytest.mark.parametrize("lights", [0, 1, 2, 4, 16])
def test_workspace_layout_covers_every_array(cap, steps, lights):
    """The render workspace (rt_capi.cpp layout_workspace) for every batch capacity the renderer
    can ask for, max_lvl 0-254 and 0-16 lights: each array lies inside the allocation the library
    makes (the sizing and the carving are one function; r02's abort was a carving that outgrew a
    separately written size), no two arrays overlap, every array is 256-B aligned and holds what
    the kernels index: queues c x 16 B, shadow pairs c x L, chain records c x steps x 16 B, the
    counters 2 x 4096 words, the work-queue slots 2 x steps x 128 words, and the batch order/cost
    arrays one entry per wave batch of the densest fused packing (>= 33 samples per batch: spp 33)."""
    total, ext = _layout(cap, steps, lights)
    L = max(lights, 1)
    need = [cap * 16] * 4 + [cap * 4, cap * 16, cap * L * 16, cap * L * 16, cap * L, cap * steps * 16,
                             cap * steps * 16, cap, 4 * 2 * 4096, 4 * 2 * 4096, 4 * 2 * steps * 128]
    nbatch = max((cap + spb - 1) // spb for spb in [(64 // s) * s for s in range(1, 65)])
    need += [4 * nbatch] * 4 + [4 * 128] + [4 * nbatch] * 2   # (+ a moving view's dilated costs and cells)
    assert len(need) == _capi.RT_WS_ARRAYS
    end = 0
    for (off, size), n in zip(ext, need):
        off, size = int(off), int(size)
        assert off % 256 == 0 and off >= end, (off, end)
        assert size >= n
        end = off + size
    assert end <= total


def test_multiframe_and_reserve_entries_refuse_without_a_device(tmp_path):
    """rt_render_frames_device and rt_scene_reserve (r05) on a host-only scene return RT_E_NODEV, and
    with a NULL scene RT_E_ARG, before touching HIP (no GPU needed)."""
    p = tmp_path / "t.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    s = R.Scene.load(str(p), device=R.RT_HOST_ONLY)
    rp = R.RenderParams(width=8, height=8, pf=1, max_lvl=1)
    with pytest.raises(R.RtError) as ei:
        s.reserve(rp, 16, 16)
    assert ei.value.code == _capi.RT_E_NODEV
    with pytest.raises(R.RtError) as ei:
        s.render_frames_device([rp, rp], 16, 16, [1, 2], 8 * 8 * 3)
    assert ei.value.code == _capi.RT_E_NODEV
    lib = _capi.lib()
    cp = rp.to_c()
    outs = (C.c_void_p * 2)(1, 2)
    assert lib.rt_render_frames_device(None, C.byref(cp), 2, 16, 16, outs, 192, None, None) == _capi.RT_E_ARG
    assert lib.rt_scene_reserve(None, C.byref(cp), 16, 16, 0) == _capi.RT_E_ARG
    assert _capi.MAX_FRAMES_PER_CALL == 8


def test_every_c_entry_is_exception_guarded():
    """No C++ exception crosses the C ABI (a failed host allocation is RT_E_NOMEM, not std::terminate in
    the host): every rt_* entry defined in the library's C-ABI sources runs its body in try/catch."""
    import os
    import re
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raytracert_amd", "csrc")
    seen = 0
    for f in ("rt_capi.cpp", "rt_comm.cpp"):
        text = open(os.path.join(src, f)).read()
        for m in re.finditer(r"^(int|void) (rt_\w+)\([^;{]*\)\s*\{\n(\s*)(\S+)", text, re.M):
            seen += 1
            assert m.group(4) == "try", f"{f}: {m.group(2)} is not wrapped in try/catch"
            body = text[m.end():text.find("\n}\n", m.end())]
            assert "catch (...)" in body, f"{f}: {m.group(2)} has no catch (...)"
    assert seen >= 50
