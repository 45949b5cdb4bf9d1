import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import graphframes_amd as gfa
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
s, d = gfa.gen_rmat(scale, 16, seed=1)
print("gen ok", flush=True)
g = gfa.Graph(s, d, 1 << scale)
print("build ok", g.info(), flush=True)
for t in range(6):
    t0 = time.time()
    st = g.step(1, stats=True)
    print("step", t + 1, round(time.time() - t0, 3), {k: round(v, 3) for k, v in st["kernel_ms"].items()}, flush=True)
