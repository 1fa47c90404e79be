"""Device JSON decode (csrc/kernels/decode.hip): bit-exact parity with the host parser on every value
it accepts, host fallback for everything unusual, and the worker's device-decode path end to end."""
import json
import urllib.error
import urllib.request

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _host(native, text: bytes, cap):
    body = b'{"request_id":"x","input_data":[' + text + b"]}"
    _, vals, n = native.parse_infer(body, cap)
    return vals, n


def _texts():
    rng = np.random.default_rng(0)
    n = 5000
    u = rng.random(n)
    s = rng.standard_normal(n).astype(np.float32)
    out = {
        "4dec_unit": ",".join("%.4f" % x for x in u),
        "7dec_signed": ",".join("%.7f" % x for x in (u * 6 - 3)),
        "repr_f32": ",".join(repr(float(x)) for x in s),
        "repr_f64": ",".join(repr(float(x)) for x in rng.random(n)),
        "ints": ",".join(str(int(x)) for x in rng.integers(-100000, 100000, n)),
        "exponents": ",".join("%.6e" % x for x in s * 10.0 ** rng.integers(-15, 15, n)),
        "spaces": ", ".join("%.3f" % x for x in u[:2000]) + " ,\n\t" + "1.5 ",
        "zeros": ",".join(["0", "-0", "0.0", "-0.000", "0e5"] * 10),
        "g17": ",".join("%.17g" % x for x in rng.random(n) * 1e3),
    }
    return {k: v.encode() for k, v in out.items()}


def test_decode_matches_host_bit_exact(native):
    from die_amd.ops import kernels as K

    texts = _texts()
    names = list(texts)
    numel = 6000
    vals, status, ntok = K.decode_json_numbers([texts[k] for k in names], numel)
    vals, status, ntok = vals.cpu().numpy(), status.cpu().numpy(), ntok.cpu().numpy()
    for i, k in enumerate(names):
        hv, hn = _host(native, texts[k], numel)
        assert ntok[i] == hn, (k, ntok[i], hn)
        if k in ("repr_f64", "g17"):
            # 17 significant digits: many tokens go to the host fallback (> 16 digits / hazard)
            assert status[i] in (0, 1)
        else:
            assert status[i] == 0, (k, status[i])
        if status[i] == 0:
            np.testing.assert_array_equal(vals[i, :hn].view(np.uint32), hv.view(np.uint32), err_msg=k)
            assert np.all(vals[i, hn:] == 0)


def test_decode_offset_table_matches_contiguous(native):
    """Staged-upload layout: samples at arbitrary arena slots located through the offset table give
    the same bits as the contiguous layout."""
    import torch
    from die_amd.ops import kernels as K

    texts = _texts()
    lst = [texts[k] for k in texts] + [None]
    a = K.decode_json_numbers(lst, 6000, text_cap=128 * 1024)
    b = K.decode_json_numbers(lst, 6000, text_cap=128 * 1024, slot_order=[7, 3, 11, 0, 5, 9, 2, 12, 8, 1])
    for x, y in zip(a, b):
        assert torch.equal(x.cpu().view(torch.int32) if x.dtype == torch.float32 else x.cpu(),
                           y.cpu().view(torch.int32) if y.dtype == torch.float32 else y.cpu())


@pytest.mark.parametrize("bad", [b"1.", b".5", b"01", b"abc", b"1,,2", b"[1]", b'"1"', b"1e", b"+1", b"--1",
                                 b"1" * 70, b"1e-50", b"3e39", b"nan", b"1 2", b"1,"])
def test_decode_flags_unusual_tokens(native, bad):
    from die_amd.ops import kernels as K

    text = b"0.5," + bad + b",0.25"
    vals, status, ntok = K.decode_json_numbers([text], 16)
    assert int(status[0]) & 1, bad


def test_decode_counts_padding_and_overflow(native):
    from die_amd.ops import kernels as K

    texts = [b"1,2,3", b"", b" ", None, b",".join([b"0.5"] * 20)]
    vals, status, ntok = K.decode_json_numbers(texts, 8)
    st = status.cpu().numpy()
    nt = ntok.cpu().numpy()
    v = vals.cpu().numpy()
    assert st[0] == 0 and nt[0] == 3 and list(v[0]) == [1, 2, 3, 0, 0, 0, 0, 0]
    assert st[1] == 0 and nt[1] == 0 and np.all(v[1] == 0)
    assert nt[2] == 0  # whitespace only: zero values (may route through the host fallback)
    assert st[3] == 0 and nt[3] == -1 and np.all(np.isnan(v[3]))  # skipped sample untouched
    assert st[4] == 2 and nt[4] == 20


def test_decode_long_text_multi_chunk(native):
    from die_amd.ops import kernels as K

    rng = np.random.default_rng(3)
    x = rng.random(150528)
    text = ",".join("%.4f" % v for v in x).encode()  # ~1 MB, ~260 chunks, tokens straddle chunk edges
    vals, status, ntok = K.decode_json_numbers([text, text], 150528)
    hv, hn = _host(native, text, 150528)
    assert int(status[0]) == 0 and int(ntok[0]) == 150528
    got = vals.cpu().numpy()
    np.testing.assert_array_equal(got[0].view(np.uint32), hv.view(np.uint32))
    np.testing.assert_array_equal(got[1], got[0])


def _post(url, body):
    req = urllib.request.Request(url + "/infer", data=body, headers={"Content-Type": "application/json"})
    try:
        return 200, json.loads(urllib.request.urlopen(req, timeout=60).read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read())


def test_worker_device_decode_matches_host_parse(native, models):
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    a = native.Worker(path, node_id="dev", engine={"device": "hip", "device_decode": True, "autotune": False})
    b = native.Worker(path, node_id="host", engine={"device": "hip", "device_decode": False, "autotune": False})
    try:
        assert a.health()["engine"]["device_decode"] is True
        assert b.health()["engine"]["device_decode"] is False
        x = r.synthetic_input(3, cfg).reshape(3, -1)
        bodies = [
            json.dumps({"request_id": "q%d" % i, "input_data": [float(v) for v in x[i]]}).encode() for i in range(3)
        ]
        bodies.append(b'{"request_id":"exotic","input_data":[1e-50, 0.5, 12345678901234567890]}')  # host fallback
        bodies.append(b'{"input_data":[1,2,3],"request_id":"order"}')
        for body in bodies:
            sa, oa = _post(a.url, body)
            sb, ob = _post(b.url, body)
            assert sa == sb == 200, (oa, ob)
            assert oa["output_data"] == ob["output_data"]
        ha = a.health()
        assert ha["device_decoded"] >= 4 and ha["decode_fallbacks"] >= 1
        for bad in [b'{"request_id":"e1","input_data":[1,abc]}', b'{"request_id":"e2","input_data":[1,2,]}',
                    b'{"request_id":"e3","input_data":[' + b",".join([b"1"] * (3 * 64 * 64 + 1)) + b"]}"]:
            sa, oa = _post(a.url, bad)
            sb, ob = _post(b.url, bad)
            assert sa == sb == 500
            assert oa["error"] == ob["error"], (oa, ob)
    finally:
        a.stop()
        b.stop()


@pytest.mark.parametrize("opts", [{"stage_slots": -1}, {"stage_slots": -1, "pipeline_depth": 1},
                                  {"exec_streams": 2}, {"stage_slots": 16, "exec_streams": 2}])
def test_worker_serving_modes_match(native, models, opts):
    """Early upload (stage_text tickets), concurrent executors and pipeline depths give the same
    answers as the default path, under concurrent load (loadgen) and for single requests."""
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    base = {"device": "hip", "autotune": False}
    a = native.Worker(path, node_id="mode", max_batch=8, engine=dict(base, max_batch=8, **opts))
    b = native.Worker(path, node_id="ref", max_batch=8, engine=dict(base, max_batch=8))
    try:
        he = a.health()["engine"]
        if opts.get("stage_slots"):
            assert he["stage_slots"] > 0
        x = r.synthetic_input(4, cfg).reshape(4, -1)
        for i in range(4):
            body = json.dumps({"request_id": "s%d" % i, "input_data": [float(v) for v in x[i]]}).encode()
            sa, oa = _post(a.url, body)
            sb, ob = _post(b.url, body)
            assert sa == sb == 200
            assert oa["output_data"] == ob["output_data"]
        numel = int(np.prod(x.shape[1:]))
        res = native.loadgen(port=a.port, connections=16, requests=400, payload="full", input_numel=numel,
                             decimals=4, seed=7, timeout_ms=30000)
        assert res["ok"] == 400 and res["failed"] == 0, res
        h = a.health()
        if opts.get("stage_slots"):
            assert h["engine"]["staged_uploads"] >= 400
    finally:
        a.stop()
        b.stop()


def _dumps_texts(n_samples, numel, seed=0):
    rng = np.random.default_rng(seed)
    x = (np.round(rng.random((n_samples, numel)), 4)).astype(np.float32)
    texts = [json.dumps([float(v) for v in row])[1:-1].encode() for row in x]  # ", " separators, repr floats
    return x, texts


def test_decode_json_dumps_payloads(native):
    from die_amd.ops import kernels as K

    x, texts = _dumps_texts(3, 12288)
    vals, status, ntok = K.decode_json_numbers(texts, 12288)
    assert status.cpu().numpy().tolist() == [0, 0, 0]
    np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint32), x.view(np.uint32))


def _identity_model(path, C=3, H=16, W=16):
    from die_amd.utils.onnx_writer import GraphBuilder

    g = GraphBuilder(name="probe")
    w = np.zeros((8, C, 1, 1), np.float32)
    for c in range(C):
        w[c, c, 0, 0] = 1.0
    g.init("w", w)
    xin = g.input("x", ["N", C, H, W])
    y = g.node("Conv", [xin, "w"], name="probe", kernel_shape=[1, 1])
    g.output(y, ["N", 8, H, W])
    g.save(path, opset=13)


def test_engine_run_text_matches_floats(native, tmp_path):
    p = str(tmp_path / "probe.onnx")
    _identity_model(p)
    e = native.Engine(p, device="hip", max_batch=4)
    x, texts = _dumps_texts(4, 3 * 16 * 16, seed=1)
    texts[2] = b"1,2,3"  # short -> zero padded
    x[2] = 0
    x[2, :3] = [1, 2, 3]
    got, st = e.run_text(texts)
    assert st.tolist() == [0, 0, 0, 0]
    ref = e.run(x)
    np.testing.assert_array_equal(got, ref)
    e.close()


def test_engine_run_text_resnet_tiny(native, models):
    path, w, cfg = models["tiny"]
    e = native.Engine(path, device="hip", max_batch=4)
    x, texts = _dumps_texts(3, 3 * 64 * 64, seed=2)
    got, st = e.run_text(texts)
    assert st.tolist() == [0, 0, 0]
    np.testing.assert_array_equal(got, e.run(x))
    e.close()


@pytest.mark.gpu
def test_engine_run_text_packed_matches_raw(native, tmp_path):
    """4-bit packed upload (device unpack -> decode) is bit-identical to the raw-text path; a batch
    may mix packed and raw (non-packable) samples, with odd and even text lengths."""
    p = str(tmp_path / "probe.onnx")
    _identity_model(p)
    e = native.Engine(p, device="hip", max_batch=8)
    assert e.text_packing
    x, texts = _dumps_texts(6, 3 * 16 * 16, seed=7)
    texts[1] = texts[1] + b" "  # odd/even length flip
    texts[3] = texts[3].replace(b", ", b",\n", 5)  # newline: not packable -> raw upload
    texts[4] = b"1,2,3"
    x[4] = 0
    x[4, :3] = [1, 2, 3]
    texts[5] = texts[5].replace(b"0.", b"0.0e0", 0) + b",1E0"  # 'E' -> raw; one extra value
    assert native.pack_nibbles(texts[3]) is None and native.pack_nibbles(texts[5]) is None
    raw, st_raw = e.run_text(texts, pack=False)
    packed, st_packed = e.run_text(texts, pack=True)
    assert st_packed.tolist() == st_raw.tolist()
    assert st_raw[:5].tolist() == [0, 0, 0, 0, 0]
    np.testing.assert_array_equal(packed, raw)
    ref = e.run(x[:5])
    np.testing.assert_array_equal(packed[:5], ref)
    e.close()


def test_decode_batch_above_one_launch(native):
    """More samples than one launch's sample table (kDecMaxB = 1024): the launcher runs passes; every
    sample (first, last, both sides of the pass boundary) decodes to its own values."""
    from die_amd.ops import kernels as K

    B = 1100
    texts = [("%d,%d.5,-%d" % (i, i % 7, i)).encode() if i % 97 else None for i in range(B)]
    vals, status, ntok = K.decode_json_numbers(texts, 4)
    v, st, nt = vals.cpu().numpy(), status.cpu().numpy(), ntok.cpu().numpy()
    for i in (0, 1, 1022, 1023, 1024, 1025, B - 1):
        if texts[i] is None:
            assert nt[i] == -1
            continue
        assert st[i] == 0 and nt[i] == 3, (i, st[i], nt[i])
        assert list(v[i]) == [float(i), (i % 7) + 0.5, -float(i), 0.0], (i, v[i])
    assert (st == 0).all()


def test_decode_long_tokens_across_lanes_and_chunks(native):
    """Tokens longer than the 32-byte register window (33-40 chars: many zeros after the point, few
    significant digits) mixed with short ones over ~30 chunks: they start in one lane's 64-byte
    region and end in the next, and straddle 4 KiB chunk boundaries (byte-wise LDS path, next-lane
    and last-token ends).  Bit-exact against the host parser."""
    from die_amd.ops import kernels as K

    rng = np.random.default_rng(11)
    parts = []
    for i in range(12000):
        v = int(rng.integers(1, 99999999))
        if i % 3 == 0:
            parts.append("0." + "0" * int(rng.integers(24, 31)) + str(v))  # 33-40 characters
        elif i % 3 == 1:
            parts.append("%.4f" % rng.random())
        else:
            parts.append("-%d.%d" % (v % 1000, v % 97))
    text = ",".join(parts).encode()
    vals, status, ntok = K.decode_json_numbers([text], len(parts))
    hv, hn = _host(native, text, len(parts))
    assert int(ntok[0]) == hn == len(parts)
    st = int(status[0])
    assert st in (0, 1)  # 1: a double-rounding hazard sent the sample to the host parser
    if st == 0:
        np.testing.assert_array_equal(vals.cpu().numpy()[0].view(np.uint32), hv.view(np.uint32))


def _pk_cases():
    t = _texts()
    rng = np.random.default_rng(5)
    extra = {
        "neg_4dec": ",".join("%.4f" % x for x in rng.random(3000) * 2 - 1),
        "dumps": ", ".join(repr(float(x)) for x in np.round(rng.random(3000), 4).astype(np.float32)),
        "mixed_len": ",".join(str(round(float(x), int(k))) for x, k in zip(rng.random(3000) * 100, rng.integers(0, 8, 3000))),
        "eight_digits": ",".join("%.8f" % x for x in rng.random(2000)) + ",16777216,16777217,99999999,0.00000001",
        "trailing_comma": "1,2,3,",
        "empty": "",
        "blank": " ",
        "lead_blank": " 1.5, -2.25,  3",
        "leading_zero": "0.5,01,0.25",
        "one": "7",
    }
    for k, v in extra.items():
        t[k] = v.encode()
    for j, bad in enumerate([b"1.", b".5", b"1,,2", b"1e", b"+1", b"--1", b"1" * 70, b"1e-50", b"3e39", b"1 2"]):
        t["bad%d" % j] = b"0.5," + bad + b",0.25"
    return t


@pytest.mark.parametrize("cap", [None, 256 * 1024])
def test_decode_packed_nibble_path_matches_raw(native, cap):
    """The nibble-level kernels (pk_count / pk_parse) that decode 4-bit packed samples give exactly the
    status, token count and value bits of the character kernels on the same texts: number shapes,
    json.dumps ", " separators, > 8 digits, exponents, blanks, and every error class (round 5)."""
    from die_amd.ops import kernels as K

    cases = _pk_cases()
    names = list(cases)
    texts = [cases[k] for k in names] + [None]
    assert native.pack_nibbles(cases["4dec_unit"]) is not None and native.pack_nibbles(cases["spaces"]) is None
    numel = 6000
    raw = [x.cpu().numpy() for x in K.decode_json_numbers(texts, numel, text_cap=cap)]
    pk = [x.cpu().numpy() for x in K.decode_json_numbers(texts, numel, text_cap=cap, packed=True)]
    for i, k in enumerate(names + ["skipped"]):
        assert pk[1][i] == raw[1][i], (k, pk[1][i], raw[1][i])
        assert pk[2][i] == raw[2][i], (k, pk[2][i], raw[2][i])
        if raw[1][i] == 0:
            np.testing.assert_array_equal(pk[0][i].view(np.uint32), raw[0][i].view(np.uint32), err_msg=k)
    st = dict(zip(names, raw[1]))
    assert st["4dec_unit"] == 0 and st["dumps"] == 0 and st["lead_blank"] == 0 and st["neg_4dec"] == 0
    assert st["trailing_comma"] & 1 and st["leading_zero"] & 1 and all(st["bad%d" % j] & 1 for j in range(10))


def test_decode_packed_long_text_multi_chunk(native):
    """A ResNet-sized packed sample (~1 MB of text, ~257 chunks, tokens straddling chunk edges) and a
    slot-permuted batch: bit-exact against the host parser."""
    from die_amd.ops import kernels as K

    rng = np.random.default_rng(9)
    text = ",".join("%.4f" % v for v in rng.random(150528)).encode()
    short = b"1,2,3"
    vals, status, ntok = K.decode_json_numbers([text, short, text], 150528, packed=True, slot_order=[2, 0, 1])
    hv, hn = _host(native, text, 150528)
    assert status.cpu().tolist() == [0, 0, 0] and ntok.cpu().tolist() == [150528, 3, 150528]
    got = vals.cpu().numpy()
    np.testing.assert_array_equal(got[0].view(np.uint32), hv.view(np.uint32))
    np.testing.assert_array_equal(got[2], got[0])
    assert list(got[1, :4]) == [1.0, 2.0, 3.0, 0.0] and not got[1, 3:].any()
