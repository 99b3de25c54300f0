"""Test helpers: run the same frames through the HIP renderer and the CPU oracle."""
import numpy as np

from rtamd import configs as cf


def frames_for(fp, first_loop: int, n: int, ro_offset: int = 0):
    ro = cf.rand_origins(n, ro_offset)
    return ro, [cf.oracle_frame_params(fp, first_loop + k, ro[k]) for k in range(n)]


def oracle_render(sd, env, W, H, frames, accum=None, x0=0, y0=0, w=None, h=None):
    import oracle as orc
    scene = orc.OracleScene(sd.tri_enc, sd.node_enc, env[0], env[1])
    return orc.render(scene, frames, W, H, x0=x0, y0=y0, w=w, h=h, accum=accum)


def gpu_render(r, sd, env, W, H, fp, ro, tile=32, rank=0, world=1, encoded=False, accum=None, loop_num=0, owner=None):
    if encoded:
        r.set_scene_encoded(sd.tri_enc, sd.node_enc)
    else:
        r.set_scene_soa(sd.soa, sd.nodes)
    r.set_env(env[0], env[1])
    r.resize(W, H, tile=tile, rank=rank, world=world)
    if owner is not None:
        r.set_tile_owners(owner)
    if accum is not None:
        r.write_accum(accum)
    r.set_loop_num(loop_num)
    r.reset_stats()
    st = r.render(fp, ro)
    return r.read_accum(), st


def bit_mismatch(a, b):
    """Fraction of pixels whose RGB float32 bit patterns differ (NaN == NaN by bits)."""
    ua = np.ascontiguousarray(a, np.float32).view(np.uint32)
    ub = np.ascontiguousarray(b, np.float32).view(np.uint32)
    diff = np.any(ua != ub, axis=-1)
    return float(diff.mean()), diff
