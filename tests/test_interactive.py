"""Interactive loop: rtamd.interactive restates Camera.h + main.cpp's loop.

CPU: camera state machine (WASDQE moves without touching the view vectors, mouse sensitivity,
the reference's pitch clamp quirk, LoopNum resets), and the loop's control flow over a recording
fake renderer (which edits reset the accumulation, randOrigin stream, display flags).  GPU: a
scripted session (moves, drags, GUI edits, zoom) displayed frame by frame equals the
oracle's frames with the same uniforms, LoopNum and randOrigin, bit for bit.
"""
import numpy as np
import pytest

from rtamd import configs as cf
from rtamd import interactive as ia
from rtamd import scene_lib as sl
from rtamd.renderer import RT_DISPLAY_GAMMA, RT_DISPLAY_TONEMAP

f32 = np.float32


def test_initial_camera_matches_frame_params():
    W, H = 1920, 1080
    cam = ia.Camera(float(f32(W) / f32(H)))
    fp = cf.frame_params(W, H)
    for k in ("front", "right", "up", "left_bottom_corner"):
        assert np.array_equal(getattr(cam, k), np.asarray(getattr(fp, k), f32)), k
    assert cam.half_h == f32(fp.half_h) and cam.half_w == f32(fp.half_w)
    assert np.array_equal(cam.position, np.array(cf.CAMERA_POSITION, f32))


def test_keyboard_moves_position_only_and_resets():
    cam = ia.Camera(2.0)
    cam.take_reset()
    front, right, up, lbc = cam.front.copy(), cam.right.copy(), cam.up.copy(), cam.left_bottom_corner.copy()
    p0 = cam.position.copy()
    dt = 0.0166
    cam.process_keyboard(ia.FORWARD, dt)
    v = f32(f32(2.5) * f32(dt))
    assert np.array_equal(cam.position, (p0 + (front * v).astype(f32)).astype(f32))
    cam.process_keyboard(ia.LEFT, dt)
    cam.process_keyboard(ia.DOWN, dt)
    exp = (p0 + (front * v).astype(f32)).astype(f32)
    exp = (exp - (right * v).astype(f32)).astype(f32)
    exp = (exp - (up * v).astype(f32)).astype(f32)
    assert np.array_equal(cam.position, exp)
    # Camera.h:83-99 never calls updateCameraVectors: the view is unchanged
    for a, b in ((cam.front, front), (cam.right, right), (cam.up, up), (cam.left_bottom_corner, lbc)):
        assert np.array_equal(a, b)
    assert cam.take_reset() and not cam.take_reset()


def test_mouse_sensitivity_and_pitch_quirk():
    cam = ia.Camera(2.0, rotation=(-90.0, 0.0, 0.0))
    cam.process_mouse_movement(10.0, -5.0)
    assert cam.yaw == f32(f32(-90.0) + f32(f32(10.0) * f32(0.1)))
    assert cam.pitch == f32(f32(0.0) + f32(f32(-5.0) * f32(0.1)))
    ref = sl.camera(float(cam.yaw), float(cam.pitch), 30.0, 2.0)
    assert np.array_equal(cam.front, ref["front"])
    cam = ia.Camera(2.0, rotation=(-90.0, 88.95, 0.0))
    cam.process_mouse_movement(0.0, 10.0)
    assert cam.pitch == f32(89.0)
    cam = ia.Camera(2.0, rotation=(-90.0, -88.95, 0.0))
    cam.process_mouse_movement(0.0, -10.0)
    assert cam.pitch == f32(89.0)  # Camera.h:124-125: a pitch below -89 becomes +89


def test_scroll_clamps_zoom():
    cam = ia.Camera(2.0)
    cam.process_mouse_scroll(100.0)
    assert cam.zoom == f32(1.0)
    cam.process_mouse_scroll(-100.0)
    assert cam.zoom == f32(45.0)
    assert cam.half_w == f32(cam.half_h * f32(2.0))


class FakeRenderer:
    """Records the loop's calls; LoopNum semantics of rt_render (main.cpp:175 LoopIncrease)."""

    def __init__(self):
        self.calls, self.loop = [], 0

    def resize(self, w, h, **_):
        self.calls.append(("resize", w, h))

    def reset(self):
        self.calls.append(("reset",))
        self.loop = 0

    def update_materials(self, first, count, texels):
        self.calls.append(("materials", first, count))

    def render(self, fp, ro):
        mi = fp.max_iterations
        if mi == -1 or self.loop < mi:
            self.loop += 1
        self.calls.append(("render", float(ro[0]), self.loop))
        return {}

    @property
    def loop_num(self):
        return self.loop

    def tonemap(self, flags):
        self.calls.append(("tonemap", flags))
        return np.zeros((1, 1, 3), np.uint8)


class FakeAsyncRenderer(FakeRenderer):
    """FakeRenderer plus the queued display of Session(frames_in_flight > 1)."""

    def __init__(self):
        super().__init__()
        self.slots, self.depth = {}, None

    def set_pipeline(self, depth):
        self.depth = depth

    def render_async(self, fp, ro):
        self.render(fp, ro)

    def tonemap_async(self, slot, flags):
        assert slot not in self.slots, "display slot reused before it was fetched"
        self.slots[slot] = (self.loop, flags)

    def display_fetch(self, slot):
        loop, flags = self.slots.pop(slot)
        return np.full((1, 1, 3), loop, np.uint8)


def test_session_frames_in_flight_returns_frames_in_order():
    """Session(frames_in_flight=D): tick k returns frame k-D+1 with its own image (the display
    queue), None while the queue fills, flush() the rest; slots never reused while queued."""
    for depth in (2, 3):
        r = FakeAsyncRenderer()
        s = ia.Session(r, 16, 16, frames_in_flight=depth)
        assert r.depth == depth
        got = [s.tick(delta_time=0.0) for _ in range(7)]
        assert got[:depth - 1] == [None] * (depth - 1)
        shown = [g for g in got if g is not None] + s.flush()
        assert [o["loop_num"] for o in shown] == list(range(1, 8))
        assert all(int(o["image"][0, 0, 0]) == o["loop_num"] for o in shown)
        assert not r.slots
    with pytest.raises(ValueError):
        ia.Session(FakeAsyncRenderer(), 16, 16, frames_in_flight=4)


def test_session_loop_resets_and_rand_stream():
    r = FakeRenderer()
    s = ia.Session(r, 64, 32)
    ro = sl.cpu_rand_origins(cf.RAND_SEED, 9)
    assert s.tick(delta_time=0.01)["loop_num"] == 1
    assert s.tick(delta_time=0.01)["loop_num"] == 2
    out = s.tick(ia.Input(keys=["w"]), delta_time=0.01)
    assert out["loop_num"] == 1 and ("reset",) in r.calls[-4:]
    assert s.tick(ia.Input(gui={"enable_tone_mapping": False}), delta_time=0.01)["loop_num"] == 2
    assert r.calls[-1] == ("tonemap", 0)
    assert s.tick(ia.Input(gui={"env_intensity": 2.0}), delta_time=0.01)["loop_num"] == 1
    # mouse: the first event only records the cursor, moves without the right button do nothing,
    # and any right-button event (even a zero offset) refreshes the camera vectors: LoopNum = 0
    assert s.tick(ia.Input(mouse=[(100, 100, False), (120, 100, False)]), delta_time=0.01)["loop_num"] == 2
    assert s.tick(ia.Input(mouse=[(120, 100, True)]), delta_time=0.01)["loop_num"] == 1
    assert s.tick(ia.Input(mouse=[(130, 90, True)]), delta_time=0.01)["loop_num"] == 1
    assert s.camera.yaw == f32(f32(cf.CAMERA_ROTATION[0]) + f32(f32(10.0) * f32(0.1)))
    renders = [c for c in r.calls if c[0] == "render"]
    assert [c[1] for c in renders] == [float(x) for x in ro[:8]]
    s.settings.enable_tone_mapping = True
    s.tick(delta_time=0.01)
    assert r.calls[-1] == ("tonemap", RT_DISPLAY_TONEMAP | RT_DISPLAY_GAMMA)


def test_session_max_iterations_and_materials():
    r = FakeRenderer()
    s = ia.Session(r, 8, 8, settings=ia.Settings(max_iterations=3))
    loops = [s.tick(delta_time=0.0)["loop_num"] for _ in range(5)]
    assert loops == [1, 2, 3, 3, 3]
    out = s.tick(ia.Input(materials=[(0, 4, cf.MATERIALS["golden"])]), delta_time=0.0)
    assert out["loop_num"] == 1 and ("materials", 0, 4) in r.calls


@pytest.mark.gpu
def test_gpu_session_matches_oracle(gpu_renderer, env_maps):
    from helpers import oracle_render
    import oracle as orc

    sd = cf.config_scene("C2")
    W, H = 48, 30
    r = gpu_renderer
    r.set_scene_soa(sd.soa, sd.nodes)
    r.set_env(env_maps[0], env_maps[1])
    s = ia.Session(r, W, H, settings=ia.Settings(max_bounce=4))
    script = [ia.Input(), ia.Input(), ia.Input(keys=["w", "d"]), ia.Input(),
              ia.Input(mouse=[(10, 10, True), (25, 4, True)]), ia.Input(gui={"enable_mis": False}),
              ia.Input(gui={"enable_tone_mapping": False}), ia.Input(camera_zoom=20.0)]
    accum = None
    for k, inp in enumerate(script):
        out = s.tick(inp, delta_time=0.05)
        frame = cf.oracle_frame_params(out["params"], out["loop_num"], out["rand_origin"])
        ref, _ = oracle_render(sd, env_maps, W, H, [frame], accum=accum)
        accum = ref
        got = r.read_accum()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), f"tick {k}"
        st = s.settings
        flags = (RT_DISPLAY_TONEMAP if st.enable_tone_mapping else 0) | \
                (RT_DISPLAY_GAMMA if st.enable_tone_mapping and st.enable_gamma_correction else 0)
        assert np.array_equal(out["image"], orc.display(ref, flags)), f"tick {k}"


@pytest.mark.gpu
@pytest.mark.parametrize("in_flight", [2, 3])
def test_gpu_session_frames_in_flight_match_oracle(gpu_renderer, env_maps, in_flight):
    """Session(frames_in_flight > 1): frames and display passes queued without waiting (the GL
    frame queue); each displayed image, fetched in_flight - 1 ticks later, equals the oracle's
    image of its own frame, through camera moves, GUI edits and a material update."""
    from helpers import oracle_render
    import oracle as orc

    sc = sl.Scene()
    for o in cf.CONFIGS["C3"].objects:
        sc.add_mesh(cf.load_mesh(o.mesh), cf.MATERIALS[o.material], o.rotate, o.translate, o.scale, o.smooth)
    sc.build_bvh(8)

    def scene_data():
        tri, nodes = sc.encode()
        return cf.SceneData("custom", sc.counts(), tri, nodes, sc.export_soa(), sc.nodes(), [])

    sd = scene_data()
    W, H = 96, 64
    r = gpu_renderer
    r.set_scene_soa(sd.soa, sd.nodes)
    r.set_env(env_maps[0], env_maps[1])
    s = ia.Session(r, W, H, settings=ia.Settings(max_bounce=4), frames_in_flight=in_flight)
    script = [ia.Input(), ia.Input(), ia.Input(), ia.Input(keys=["w", "d"]), ia.Input(), ia.Input(),
              ia.Input(mouse=[(10, 10, True), (25, 4, True)]), ia.Input(),
              ia.Input(materials=[(0, 50000, cf.MATERIALS["golden"])]), ia.Input(),
              ia.Input(gui={"enable_tone_mapping": False}), ia.Input()]
    shown = []
    for inp in script:
        out = s.tick(inp, delta_time=0.05)
        if out is not None:
            shown.append(out)
    shown += s.flush()
    assert len(shown) == len(script)
    # the oracle replays the frames in order; the material update re-encodes the scene as the
    # renderer's rt_update_materials does (RefreshTriangleMaterial)
    accum, sdk = None, sd
    for k, out in enumerate(shown):
        if k == 8:
            sc.set_material(0, 50000, cf.MATERIALS["golden"])
            sdk = scene_data()
        frame = cf.oracle_frame_params(out["params"], out["loop_num"], out["rand_origin"])
        accum, _ = oracle_render(sdk, env_maps, W, H, [frame], accum=accum)
        assert np.array_equal(out["image"], orc.display(accum, out["display_flags"])), f"tick {k}"
    s.r.set_pipeline(1)
