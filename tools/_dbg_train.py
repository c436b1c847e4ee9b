import sys, numpy as np, torch
sys.path.insert(0, "tests"); sys.path.insert(0, "rag-snvbert_amd"); sys.path.insert(0, ".")
from conftest import load_golden
import test_gpu_train as T
from src.engine import engine_for
g, cfg, m = T._train_model("train_tiny")
x = T._train_inputs(g)
f = load_golden("fwd_tiny")
for mod in m.modules():
    if isinstance(mod, torch.nn.BatchNorm1d):
        mod.eval()
with torch.no_grad():
    out_t = m(x)
    m.eval(); eng = engine_for(m); eng.set_dtype(torch.bfloat16)
    out_e = m(x)
    eng.set_dtype(torch.float32)
    out_f = m(x)
ref = f["can_probs_h1"]
print("rag inputs equal fwd_tiny canonical? ", np.abs(f["Ican_h1"]).sum())
for name, o in (("train", out_t), ("eval bf16", out_e), ("eval f32", out_f)):
    print(name, "max|p1 - ref_eval|", float(np.abs(o[0].float().cpu().numpy() - ref).max()),
          "max|p1 - ref_train|", float(np.abs(o[0].float().cpu().numpy() - g["probs_h1"]).max()))
print("ref eval vs ref train", float(np.abs(ref - g["probs_h1"]).max()))
