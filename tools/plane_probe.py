import sys, os, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch, bench
tsa = bench.load_pkg()
import tsa_amd.synth as synth
L = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
p = tsa.TsaParams.default(score_bits=16)
a, b, c = synth.triple(0, L, L, L)
seqs, offs = tsa.pack_batch([(a, b, c)])
ds, do = torch.from_numpy(seqs).cuda(), torch.from_numpy(offs).cuda()
sc = torch.zeros(1, dtype=torch.int32, device="cuda")
os.environ["TSA_PENCIL_MODE"] = "plane"
ws = tsa.workspace_size(1, L, L, L, p, "plane")
dw = torch.empty(ws, dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
for r in range(3):
    torch.cuda.synchronize(); t0 = time.time()
    tsa.score_batch_async(ds.data_ptr(), do.data_ptr(), 1, L, L, L, sc.data_ptr(), dw.data_ptr(), ws, st.cuda_stream, p, "plane")
    torch.cuda.synchronize(); print(L, "plane ms", round((time.time() - t0) * 1e3, 2), "score", int(sc.item()), flush=True)
