"""CPU checks of the prune_tx_2D restatement (oracle/oracle_txfeat.c): the
neural-net evaluation (av1_nn_predict_c, av1/encoder/ml.c:31-70), the sorting
networks (av1/encoder/sorting_network.h) and the whole per-block decision
(tx_search.c:1487-1641) against an independent numpy float32 statement, on
the reference's own models and thresholds (parsed from
av1/encoder/tx_prune_model_weights.h and tx_search.c into
tests/golden/ref_tables.json)."""
import json
import os

import numpy as np
import pytest

import _oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
T = json.load(open(os.path.join(HERE, "golden", "ref_tables.json")))
NN, TH = T["tx_type_nn"], T["prune_2d_thresholds"]
TABLE2D = T["tx_type_table_2d"]
TXW = [4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64]
TXH = [4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16]
MODEL_SIZES = [s for s in range(19) if NN["hor"][s] is not None]
f32 = np.float32


def py_nn(x, cfg, reduce_prec=True):
    inp = [f32(v) for v in x[:cfg["num_inputs"]]]
    for layer, nh in enumerate(cfg["hidden"]):
        w, b = cfg["weights"][layer], cfg["bias"][layer]
        out = []
        for node in range(nh):
            val = f32(b[node])
            for i in range(len(inp)):
                val = f32(val + f32(f32(w[node * len(inp) + i]) * inp[i]))
            out.append(val if val > 0 else f32(0))
        inp = out
    w, b = cfg["weights"][-1], cfg["bias"][-1]
    res = []
    for node in range(cfg["num_outputs"]):
        val = f32(b[node])
        for i in range(len(inp)):
            val = f32(val + f32(f32(w[node * len(inp) + i]) * inp[i]))
        res.append(val)
    if reduce_prec:
        inv = f32(1.0 / 512)
        res = [f32(f32(int(float(f32(v * f32(512))) + 0.5)) * inv) for v in res]
    return np.array(res, np.float32)


def approx_exp(y):
    a = f32(f32(1 << 23) / f32(0.69314718056))
    i = np.int32(int(f32(y * a)) + ((127 << 23) - 60801))
    return i.view(np.float32)


def py_softmax16(v):
    mx = v[0]
    for t in v[1:]:
        mx = mx if mx > t else t
    out, s = [], f32(0)
    for t in v:
        d = f32(t - mx)
        e = approx_exp(d if d > f32(-10) else f32(-10))
        out.append(e)
        s = f32(s + e)
    return [f32(e / s) for e in out]


def py_sort(k, v, n):
    k, v = list(k), list(v)
    for i, j in T["sort_network_%d" % n]:
        ge = k[i] >= k[j]
        k[i], k[j] = (k[i], k[j]) if ge else (k[j], k[i])
        v[i], v[j] = (v[i], v[j]) if ge else (v[j], v[i])
    return k, v


def py_prune_one(hf, vf, hor, ver, thresh, mode, mask):
    hs, vs = py_nn(hf, hor), py_nn(vf, ver)
    raw = py_softmax16([f32(vs[i] * hs[j]) for i in range(4) for j in range(4)])
    max_i, max_s, s, allow, cnt = 0, f32(0), f32(0), 0, 0
    allowed, sc = [255] * 16, [f32(-1)] * 16
    for t in range(16):
        if not mask & (1 << TABLE2D[t]):
            continue
        if raw[t] > max_s:
            max_s, max_i = raw[t], t
        if raw[t] >= thresh:
            allow |= 1 << TABLE2D[t]
            s = f32(s + raw[t])
            sc[cnt], allowed[cnt] = raw[t], TABLE2D[t]
            cnt += 1
    if not allow & (1 << TABLE2D[max_i]):
        return allow | (1 << TABLE2D[max_i]), list(TABLE2D)
    sc, allowed = py_sort(sc, allowed, 8 if cnt <= 8 else 16)
    if mode >= 4:
        temp, ratio, n, t = f32(0), f32(0), 0, 0
        inv = f32(f32(100) / s)
        while t < cnt:
            if float(ratio) > 30.0 and n >= 2:
                break
            temp = f32(temp + sc[t])
            ratio = f32(temp * inv)
            n += 1
            t += 1
        for u in range(t, cnt):
            allow &= ~(1 << allowed[u])
    return allow, allowed


def test_tables_shape():
    assert MODEL_SIZES == [0, 1, 2, 5, 6, 7, 8, 13, 14]
    for s in MODEL_SIZES:
        hn = TXW[s] if TXW[s] <= 8 else TXW[s] // 2
        vn = TXH[s] if TXH[s] <= 8 else TXH[s] // 2
        assert NN["hor"][s]["num_inputs"] == hn and NN["ver"][s]["num_inputs"] == vn
        assert NN["hor"][s]["num_outputs"] == 4 and TH[s] is not None
    assert sorted(TABLE2D) == list(range(16))


@pytest.mark.parametrize("s", MODEL_SIZES)
@pytest.mark.parametrize("d", ["hor", "ver"])
def test_nn_predict_matches_python(s, d):
    rng = np.random.default_rng(s * 2 + (d == "ver"))
    cfg = NN[d][s]
    c = O.nn_config(cfg)
    for _ in range(40):
        x = rng.random(cfg["num_inputs"]).astype(np.float32)
        for rp in (True, False):
            np.testing.assert_array_equal(O.nn_predict(x, c, rp), py_nn(x, cfg, rp))


@pytest.mark.parametrize("n", [8, 16])
def test_sort_networks(n):
    rng = np.random.default_rng(n)
    for trial in range(200):
        k = rng.random(n).astype(np.float32)
        if trial % 3 == 0:  # ties
            k = np.round(k * 4).astype(np.float32) / 4
        v = np.arange(n, dtype=np.int32)
        ok, ov = O.sort_fi32(k, v, n)
        pk, pv = py_sort(k, v, n)
        np.testing.assert_array_equal(ok, np.array(pk, np.float32))
        np.testing.assert_array_equal(ov, np.array(pv, np.int32))
        assert (np.diff(ok) <= 0).all()


@pytest.mark.parametrize("s", MODEL_SIZES)
@pytest.mark.parametrize("set_type,mode", [(5, 1), (5, 3), (4, 2), (4, 4), (4, 5), (5, 4)])
def test_prune_matches_python(s, set_type, mode):
    if set_type == 5 and s == 2:
        pytest.skip("16x16 never uses EXT_TX_SET_ALL16 (threshold row has 10 entries)")
    bw, bh = TXW[s], TXH[s]
    rng = np.random.default_rng(s * 100 + set_type * 10 + mode)
    res = rng.integers(-60, 61, size=(bh * 4, bw * 4)).astype(np.int16)
    res[:bh, :bw] = 0  # an all-zero block: the equal-energy features
    masks = rng.integers(1, 1 << 16, size=16).astype(np.uint16)
    masks[0] = 0xFFFF
    ag = [None, (4, 1), (6, 3), (9, 6), (9, 6), (12, 9)][mode][0 if set_type == 5 else 1]
    out, maps = O.prune_tx_2d(res, bw, bh, set_type, mode, TH[s], NN["hor"][s], NN["ver"][s],
                              masks)
    hf, vf = O.tx_prune_features(res, bw, bh)
    for b in range(16):
        exp_mask, exp_map = py_prune_one(hf[b], vf[b], NN["hor"][s], NN["ver"][s],
                                         f32(TH[s][ag]), mode, int(masks[b]))
        assert int(out[b]) == exp_mask, b
        assert list(maps[b]) == exp_map, b
        assert out[b] != 0


def test_prune_passthrough():
    res = np.ones((16, 16), np.int16)
    for args in ((3, 1, TH[0], NN["hor"][0], NN["ver"][0]),   # other tx set type
                 (5, 0, TH[0], NN["hor"][0], NN["ver"][0]),   # pruning off
                 (5, 1, None, None, None)):                    # no model for the size
        out, maps = O.prune_tx_2d(res, 4, 4, *args, allowed_default=0x0F0F)
        assert (out == 0x0F0F).all()
        assert (maps == np.arange(16)).all()
