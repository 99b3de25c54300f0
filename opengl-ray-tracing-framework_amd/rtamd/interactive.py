"""The reference's interactive render loop, headless.

``Camera`` restates src/core/Camera.h (fp32 like glm::vec3): WASDQE moves the position without
touching the view vectors (Camera.h:83-99), right-button mouse drags turn yaw/pitch through
updateCameraVectors (Camera.h:115-131, :160-174, with the reference's pitch clamp that sends
pitch < -89 to +89), zoom / screen ratio / GUI edits call Refresh.  Every one of these sets
LoopNum = 0, which restarts the progressive accumulation.

``Session`` restates the body of main.cpp's render loop (main.cpp:165-253): mouse events from
the previous poll, processInput (main.cpp:267-287), OnGUI's setting and material edits
(main.cpp:329-420, each resetting LoopNum), LoopIncrease under maxIterations, one frame of the
path tracer with randOrigin = 674764 * (rand()/RAND_MAX + 1) (main.cpp:190), then the display
pass (tone mapping + gamma or the screen blit, main.cpp:202-228) read back as 8-bit RGB.  GUI,
window and GL plumbing stay out of scope; this is the loop a windowing front end drives.
"""
from __future__ import annotations

import dataclasses
import time
from typing import Dict, Iterable, Optional, Sequence

import numpy as np

from . import configs as cf
from . import scene_lib as sl
from .renderer import RT_DISPLAY_GAMMA, RT_DISPLAY_TONEMAP, FrameParams, Renderer

f32 = np.float32

# Camera.h:10-24
FORWARD, BACKWARD, LEFT, RIGHT, UP, DOWN = range(6)
SPEED = f32(2.5)
SENSITIVITY = f32(0.1)
ZOOM = f32(30.0)
# main.cpp:267-282: key -> Camera_Movement, polled in this order
KEYS = (("W", FORWARD), ("S", BACKWARD), ("A", LEFT), ("D", RIGHT), ("Q", UP), ("E", DOWN))


class Camera:
    """src/core/Camera.h.  ``loop_reset`` records the LoopNum = 0 writes since the last take."""

    def __init__(self, screen_ratio: float, position=cf.CAMERA_POSITION, rotation=cf.CAMERA_ROTATION,
                 zoom: float = float(ZOOM)):
        self.position = np.array(position, f32)
        self.rotation = np.array(rotation, f32)
        self.zoom = f32(zoom)
        self.screen_ratio = f32(screen_ratio)
        self.movement_speed = SPEED
        self.mouse_sensitivity = SENSITIVITY
        self.loop_reset = False
        self._update_vectors()  # the constructor's glm::rotate result is overwritten here (Camera.h:80)

    # Camera.h:160-174
    def _update_vectors(self) -> None:
        self.yaw, self.pitch = f32(self.rotation[0]), f32(self.rotation[1])
        c = sl.camera(float(self.yaw), float(self.pitch), float(self.zoom), float(self.screen_ratio))
        self.front, self.right, self.up = c["front"], c["right"], c["up"]
        self.left_bottom_corner = c["left_bottom_corner"]
        self.half_h, self.half_w = f32(c["half_h"]), f32(c["half_w"])
        self.loop_reset = True

    def process_keyboard(self, direction: int, delta_time: float) -> None:  # Camera.h:83-99
        velocity = f32(self.movement_speed * f32(delta_time))
        vec = {FORWARD: self.front, BACKWARD: self.front, LEFT: self.right, RIGHT: self.right,
               UP: self.up, DOWN: self.up}[direction]
        step = (vec * velocity).astype(f32)
        if direction in (FORWARD, RIGHT, UP):
            self.position = (self.position + step).astype(f32)
        else:
            self.position = (self.position - step).astype(f32)
        self.loop_reset = True

    def process_mouse_movement(self, xoffset: float, yoffset: float, constrain_pitch: bool = True) -> None:
        xoffset = f32(f32(xoffset) * self.mouse_sensitivity)  # Camera.h:115-131
        yoffset = f32(f32(yoffset) * self.mouse_sensitivity)
        yaw = f32(self.yaw + xoffset)
        pitch = f32(self.pitch + yoffset)
        if constrain_pitch:
            if pitch > f32(89.0):
                pitch = f32(89.0)
            if pitch < f32(-89.0):
                pitch = f32(89.0)  # sic: the reference clamps a low pitch to +89
        self.rotation = np.array([yaw, pitch, 0.0], f32)
        self._update_vectors()

    def process_mouse_scroll(self, yoffset: float) -> None:  # Camera.h:133-144 (unbound in main.cpp:320-322)
        zoom = f32(self.zoom - f32(yoffset))
        self.zoom = f32(min(max(zoom, f32(1.0)), f32(45.0)))
        self.half_h = f32(sl.camera(float(self.yaw), float(self.pitch), float(self.zoom), float(self.screen_ratio))["half_h"])
        self.half_w = f32(self.half_h * self.screen_ratio)
        self.left_bottom_corner = (self.front - self.half_w * self.right - self.half_h * self.up).astype(f32)
        self.loop_reset = True

    def process_screen_ratio(self, width: int, height: int) -> None:  # Camera.h:146-149
        self.screen_ratio = f32(f32(width) / f32(height))
        self._update_vectors()

    def refresh(self) -> None:  # Camera.h:155-157
        self._update_vectors()

    def take_reset(self) -> bool:
        r, self.loop_reset = self.loop_reset, False
        return r


@dataclasses.dataclass
class Settings:
    """The GUI-editable render settings (src/core/RenderSettings.h:81-90)."""
    enable_mis: bool = True
    enable_env_map: bool = True
    enable_tone_mapping: bool = True
    enable_gamma_correction: bool = True
    enable_bsdf: bool = True
    env_intensity: float = 1.0
    env_angle: float = 0.0
    max_bounce: int = 8
    max_iterations: int = 3000


# OnGUI controls that restart the accumulation (main.cpp:343-368, :408); tone mapping / gamma
# only change the display pass (main.cpp:373-374)
RESETTING = {"enable_env_map", "env_intensity", "env_angle", "enable_mis", "max_bounce", "max_iterations",
             "enable_bsdf"}


@dataclasses.dataclass
class Input:
    """What one poll of the window delivers: held keys, cursor positions seen since the last
    frame (with the right-button state of each), GUI edits, an optional framebuffer resize."""
    keys: Iterable[str] = ()
    mouse: Sequence[tuple] = ()                 # (xpos, ypos, right_button_down)
    gui: Dict[str, object] = dataclasses.field(default_factory=dict)
    camera_position: Optional[Sequence[float]] = None   # InputFloat3 "Camera Position"
    camera_rotation: Optional[Sequence[float]] = None   # InputFloat3 "Camera Rotation"
    camera_zoom: Optional[float] = None                 # SliderFloat "Camera Zoom"
    materials: Sequence[tuple] = ()             # (first_triangle, count, sl.Material): setDirty()
    resize: Optional[tuple] = None              # (width, height)


class Session:
    """main.cpp's render loop over a Renderer that already holds the scene and environment."""

    def __init__(self, renderer: Renderer, width: int, height: int, settings: Optional[Settings] = None,
                 camera: Optional[Camera] = None, rand_seed: int = cf.RAND_SEED, max_frames: int = 1 << 16,
                 frames_in_flight: int = 1):
        """frames_in_flight > 1: the GL driver's frame queue (glfwSwapBuffers does not wait for the
        frame, main.cpp:251): tick() queues its frame and display pass without waiting
        (rt_set_pipeline, rt_tonemap_async) and returns the frame displayed frames_in_flight - 1
        ticks earlier (None while the queue fills; flush() returns the rest).  Images unchanged.
        (The library overlaps at most two render calls; a third queued frame deepens the display
        queue only.)"""
        if not 1 <= frames_in_flight <= 3:
            raise ValueError("frames_in_flight must be 1, 2 or 3")
        self.r = renderer
        self.in_flight = frames_in_flight
        self._queued = []  # (tick result, display slot) of frames whose image is not fetched yet
        if frames_in_flight > 1 or hasattr(renderer, "set_pipeline"):
            self.r.set_pipeline(frames_in_flight)
        self.settings = settings or Settings()
        self.width, self.height = width, height
        self.camera = camera or Camera(float(f32(width) / f32(height)))
        self.r.resize(width, height)
        self.r.reset()
        self.camera.take_reset()
        # GetCPURandom() stream: one randOrigin per displayed frame (main.cpp:190)
        self._rand = sl.cpu_rand_origins(rand_seed, max_frames)
        self.frame = 0
        self.first_mouse = True                               # RenderSettings.h:29-31
        self.last_x, self.last_y = f32(1024 / 2.0), f32(512 / 2.0)
        self.last_time: Optional[float] = None

    # main.cpp:296-318
    def _mouse(self, xpos: float, ypos: float, rmb: bool) -> None:
        xpos, ypos = f32(xpos), f32(ypos)
        if self.first_mouse:
            self.last_x, self.last_y = xpos, ypos
            self.first_mouse = False
        xoffset, yoffset = f32(xpos - self.last_x), f32(self.last_y - ypos)
        self.last_x, self.last_y = xpos, ypos
        if rmb:
            self.camera.process_mouse_movement(xoffset, yoffset)

    def frame_params(self) -> FrameParams:
        c, s = self.camera, self.settings
        return FrameParams(position=c.position, front=c.front, right=c.right, up=c.up,
                           left_bottom_corner=c.left_bottom_corner, half_h=float(c.half_h), half_w=float(c.half_w),
                           enable_mis=s.enable_mis, enable_env_map=s.enable_env_map, enable_bsdf=s.enable_bsdf,
                           env_intensity=s.env_intensity, env_angle=s.env_angle, max_bounce=s.max_bounce,
                           max_iterations=s.max_iterations)

    def tick(self, inp: Optional[Input] = None, delta_time: Optional[float] = None, display: bool = True) -> dict:
        """One pass of the render loop; returns the frame's uniforms, LoopNum and the 8-bit image."""
        inp = inp or Input()
        now = time.perf_counter()
        if delta_time is None:  # main.cpp:166-169
            delta_time = 0.0 if self.last_time is None else now - self.last_time
        self.last_time = now
        if inp.resize is not None:  # framebuffer_size_callback (main.cpp:289-294)
            self.width, self.height = inp.resize
            self.camera.process_screen_ratio(self.width, self.height)
            self.r.resize(self.width, self.height)
        for x, y, rmb in inp.mouse:
            self._mouse(x, y, rmb)
        held = {k.upper() for k in inp.keys}
        for key, direction in KEYS:  # processInput
            if key in held:
                self.camera.process_keyboard(direction, delta_time)
        reset = False
        for name, value in inp.gui.items():  # OnGUI
            if not hasattr(self.settings, name):
                raise KeyError(f"unknown setting {name!r}")
            setattr(self.settings, name, value)
            reset |= name in RESETTING
        if inp.camera_position is not None:
            self.camera.position = np.array(inp.camera_position, f32)
            self.camera.refresh()
        if inp.camera_rotation is not None:
            self.camera.rotation = np.array(inp.camera_rotation, f32)
            self.camera.refresh()
        if inp.camera_zoom is not None:
            self.camera.zoom = f32(inp.camera_zoom)
            self.camera.refresh()
        for first, count, mat in inp.materials:  # setDirty(): RefreshTriangleMaterial + LoopNum = 0
            self.r.update_materials(first, count, mat.texels())
            reset = True
        if self.camera.take_reset() or reset:
            self.r.reset()
        fp = self.frame_params()
        ro = self._rand[self.frame:self.frame + 1]
        self.frame += 1
        # LoopIncrease under maxIterations happens inside (main.cpp:175)
        if self.in_flight > 1:
            self.r.render_async(fp, ro)
        else:
            self.r.render(fp, ro)
        out = {"params": fp, "loop_num": self.r.loop_num, "rand_origin": float(ro[0]), "delta_time": delta_time}
        s = self.settings
        flags = (RT_DISPLAY_TONEMAP if s.enable_tone_mapping else 0) | \
                (RT_DISPLAY_GAMMA if s.enable_tone_mapping and s.enable_gamma_correction else 0)
        out["display_flags"] = flags
        if self.in_flight == 1:
            if display:
                out["image"] = self.r.tonemap(flags)
            return out
        slot = None
        if display:
            slot = self.frame % 4  # at most 3 queued: a slot is fetched before it is reused
            self.r.tonemap_async(slot, flags)
        self._queued.append((out, slot))
        return self._fetch_oldest() if len(self._queued) >= self.in_flight else None

    def _fetch_oldest(self) -> dict:
        out, slot = self._queued.pop(0)
        if slot is not None:
            out["image"] = self.r.display_fetch(slot)
        return out

    def flush(self) -> list:
        """The queued frames' results, oldest first (frames_in_flight > 1)."""
        done = []
        while self._queued:
            done.append(self._fetch_oldest())
        return done
