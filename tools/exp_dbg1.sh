# per-pass debug output of one-frame calls (RT_DEBUG_PASSES), single group (development aid)
set -e
cd /root/repo
mkdir -p gpurun_out/dbg1
cat > /tmp/dbg1.py <<'PY'
import sys
sys.path.insert(0, "opengl-ray-tracing-framework_amd")
from rtamd import configs as cf
from rtamd.renderer import Renderer
sd = cf.config_scene("C3"); W, H = 1920, 1080
r = Renderer(0); r.set_scene_soa(sd.soa, sd.nodes); r.set_env(*cf.load_env()); r.resize(W, H)
fp = cf.frame_params(W, H); ro = cf.rand_origins(8)
r.set_pipeline(2)
r.order_work(fp, ro[:1])
for k in range(3):
    print("=== call", k, file=sys.stderr, flush=True)
    r.render(fp, ro[k:k+1])
PY
RT_DEBUG_PASSES=1 timeout -k 10 120 python3 /tmp/dbg1.py > gpurun_out/dbg1/log.txt 2>&1
tail -60 gpurun_out/dbg1/log.txt
