"""SSSP round counts per agent (the debug status word: rounds << 8) of a config's batch, and the
launch time with and without the debug outputs.  Diagnostic only.
    python tools/rounds_probe.py CONFIG ENVS"""
import sys, os, time
sys.path.insert(0, 'spatial-intention-maps_amd')
import numpy as np, torch
from simaps import batch, synthetic, _lib
cfg = sys.argv[1]; E = int(sys.argv[2])
scenes = [synthetic.make_scene(cfg, e) for e in range(E)]
b = batch.StateBatch(scenes)
st = torch.zeros(b.N, dtype=torch.int32, device='cuda')
out = b.alloc_state()
for rep in range(3):
    b.render(out, debug={'status': st})
    torch.cuda.synchronize()
    r = st.cpu().numpy() >> 8
    print(os.environ.get('SIMAPS_LIB', 'prod')[-20:], cfg, 'rounds: max', r.max(), 'hist', np.bincount(r)[:12].tolist(), 'argmax', np.argsort(-r)[:6].tolist())
t = time.time()
def timeit(**kw):
    for _ in range(3): b.render(out, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50): b.render(out, **kw)
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 50 * 1e3
print('us/launch plain %.1f  with status %.1f' % (timeit(), timeit(debug={'status': st})))
dbg = b.alloc_debug()
print('us/launch with full debug %.1f' % timeit(debug=dbg))
