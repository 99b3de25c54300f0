"""rtamd — MI355X-native path tracer with the rendering behaviour of
georgehuan1994/OpenGL-Ray-Tracing-Framework's fragment-shader render loop.

Host scene preparation: ``rtamd.scene_lib`` (librtscene.so, include/rt_scene.h).
GPU path tracer:        ``rtamd.renderer`` (librtamd.so, include/rt_abi.h).
Reference scene configs: ``rtamd.configs``.
"""
