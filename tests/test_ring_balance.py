"""Load shares of the gateway's consistent-hash ring at N workers.

The multi-GPU headline runs every rank's gateway over every rank's worker; the ring (FNV-1a,
"addr#i" virtual nodes, 150 each: /root/reference/src/consistent_hash.cpp:6-45,
/root/reference/include/consistent_hash.h:12) is kept bit-identical, so the busiest worker's share
bounds the job's throughput.  These tests pin the analysis behind bench.py's deployment choices
(parallel/ring_balance.py): balanced worker ports + scrambled request numbers."""
import random

import numpy as np
import pytest


def _names(ports):
    return ["127.0.0.1:%d" % p for p in ports]


def test_arc_shares_match_native_routing(native):
    from die_amd.parallel import ring_balance as rb

    names = _names([20101, 20377, 21003, 21950])
    arcs = rb.arc_shares(names)
    assert abs(arcs.sum() - 1.0) < 1e-9
    rng = random.Random(1)
    ids = ["%032x" % rng.getrandbits(128) for _ in range(20000)]
    routed = rb.route_shares(names, ids)
    np.testing.assert_allclose(routed, arcs, atol=0.015)  # uniform keys: shares = arcs


def test_arbitrary_ports_and_sequential_ids_are_unbalanced(native):
    """What the bench measured before: ephemeral ports, ids r<rank>_0000000000.. in order."""
    from die_amd.parallel import ring_balance as rb

    rng = random.Random(0)
    effs = []
    for _ in range(6):
        names = _names(rng.sample(range(32768, 61000), 8))
        ids = [x for k in range(8) for x in rb.request_ids("r%d_" % k, 500, scramble=False)]
        effs.append(rb.predict(names, ids)["efficiency"])
    assert np.median(effs) < 0.8, effs  # the busiest worker gets > 1.25x its fair share


@pytest.mark.parametrize("world", [2, 4, 8])
def test_balanced_ports_with_scrambled_ids(native, world):
    from die_amd.parallel import ring_balance as rb

    ports = rb.balanced_ports(world, range(20000, 22000), seed=world)
    assert len(set(ports)) == world and all(20000 <= p < 22000 for p in ports)
    names = _names(ports)
    assert rb.arc_shares(names).max() * world <= 1.06
    ids = [x for k in range(world) for x in rb.request_ids("r%d_" % k, 10000 // world)]
    pred = rb.predict(names, ids)
    assert pred["efficiency"] >= 0.9, pred
    print(world, ports, pred)


def test_scrambled_ids_match_the_load_generator(native):
    """request_ids() must print exactly what csrc/serve/loadgen.cpp sends (scramble_ids)."""
    import json
    import threading
    from http.server import BaseHTTPRequestHandler, HTTPServer

    from die_amd.parallel import ring_balance as rb

    seen = []

    class H(BaseHTTPRequestHandler):
        def do_POST(self):
            body = self.rfile.read(int(self.headers["Content-Length"]))
            seen.append(json.loads(body)["request_id"])
            out = b'{"ok":1}'
            self.send_response(200)
            self.send_header("Content-Length", str(len(out)))
            self.end_headers()
            self.wfile.write(out)

        def log_message(self, *a):
            pass

    srv = HTTPServer(("127.0.0.1", 0), H)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    try:
        res = native.loadgen(port=srv.server_address[1], connections=1, requests=20, payload="ref", id_prefix="r3_",
                             scramble_ids=True)
        assert res["ok"] == 20
    finally:
        srv.shutdown()
    # the "ref" payload prints the number unpadded (like the reference's "req_N"); "full" and
    # "verify" bodies carry the fixed 10 digits request_ids() returns
    assert seen == ["r3_%d" % int(x[3:]) for x in rb.request_ids("r3_", 20)]


def test_scramble_is_a_bijection():
    """the id scramble must be injective (splitmix64(i) % 10^10 was not): the Feistel map
    permutes [0, 10^10); checked exhaustively on a window and by inverting a sample."""
    from die_amd.parallel import ring_balance as rb

    n = 300000
    xs = [rb.scramble_id(i) for i in range(n)]
    assert len(set(xs)) == n and all(0 <= x < 10 ** 10 for x in xs)
    half = 10 ** 5

    def unscramble(y):  # run the 4 rounds backwards
        left, right = divmod(y, half)
        for k in reversed(range(4)):
            left, right = (right - rb.splitmix64(left * 4 + k) % half) % half, left
        return left * half + right

    for i in (0, 1, 99999, 123456789, 10 ** 10 - 1):
        assert unscramble(rb.scramble_id(i)) == i


def test_reference_layout_prediction(native):
    """bench.py reports the ring the reference's own deployment would get (ports 8001.., sequential
    req_<i> ids) next to the balanced one."""
    from die_amd.parallel import ring_balance as rb

    r = rb.reference_layout(3, 3000)
    assert r["ports"] == [8001, 8002, 8003] and abs(sum(r["shares"]) - 1.0) < 1e-6
    assert r["max_over_fair"] >= 1.0
