"""Shared synthetic block-tail case of tools/tailw_micro.py / tailw_diag.py."""
import torch

from src import kernels as K

D = 384
dev, bf = "cuda", torch.bfloat16
F = torch.nn.functional


def case(M, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    r = lambda *s, sc=1.0: (sc * torch.randn(*s, generator=g)).to(dev)
    x, att = r(M, D).to(bf), r(M, D, sc=0.5).to(bf)
    w_o, w1 = (r(D, D) / D ** 0.5).to(bf), (r(4 * D, D) / D ** 0.5).to(bf)
    w2 = r(D, 4 * D) / (4 * D) ** 0.5
    b_o, b1, b2 = r(D, sc=0.1), r(4 * D, sc=0.1), r(D, sc=0.1)
    g1, be1 = 1 + r(D, sc=0.2), r(D, sc=0.1)
    gf, bff = 1 + r(4 * D, sc=0.2), r(4 * D, sc=0.1)
    g2, be2 = 1 + r(D, sc=0.2), r(D, sc=0.1)
    w2g, b2g, _ = K.fold_layernorm(w2, b2, gf, bff, bf)
    vec = K.ffn_vec(b1, b2g, w2g, g2, be2)
    return dict(x=x, att=att, w_o=w_o, w1=w1, w2=w2, w2g=w2g, b_o=b_o, b1=b1, b2=b2, g1=g1, be1=be1, gf=gf,
                bff=bff, g2=g2, be2=be2, vec=vec)


def ref(c):
    x1 = F.layer_norm(c["x"].double() + c["att"].double() @ c["w_o"].double().T + c["b_o"].double(), (D,),
                      c["g1"].double(), c["be1"].double(), 1e-5)
    h = F.leaky_relu(x1 @ c["w1"].double().T + c["b1"].double(), 0.1)
    hn = F.layer_norm(h, (4 * D,), c["gf"].double(), c["bff"].double(), 1e-5)
    f = F.leaky_relu(hn @ c["w2"].double().T + c["b2"].double(), 0.1)
    return F.layer_norm(x1 + f, (D,), c["g2"].double(), c["be2"].double(), 1e-5)


def run(c, ts, wide):
    y = c["x"].clone()
    K.set_option("tail_wide", wide)
    K.tail_forward(c["att"], y, ts, c["b_o"], c["g1"], c["be1"], c["vec"])
    K.set_option("tail_wide", 0)
    return y


