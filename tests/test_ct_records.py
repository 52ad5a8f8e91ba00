"""Host-side checks of the conntrack record helpers the fused stage A relies on
(polycube_amd/csrc/devchain.h, compiled here with g++: the helpers are PCN_HD).

- ct_bucket(h, 2^k - 1) equals h % (2^k - 1): the Mersenne fold that replaced the
  64-bit division in the key buckets (every kernel computes buckets with it).
- A record built with placeholder stale ports and then completed by ct_rec_restale
  equals the record built with the true stale ports (ports word, rev bits, key
  bucket), for every record kind a frame without ports of its own can have: what
  conntrack.hip ct_stale_fix does to the records stage A marks."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r'''
#include <cstdio>
#include <cstdlib>
#include <random>
#include "devchain.h"
using namespace pcn;
int main() {
  std::mt19937_64 g(12345);
  long bad = 0, n = 0;
  for (uint32_t k = 8; k <= 30; ++k) {
    const uint32_t s = (1u << k) - 1;
    const uint64_t edge[] = {0, s, uint64_t(s) + 1, 2ull * s, 2ull * s + 1, ~0ull, ~0ull - 1, uint64_t(s) * s};
    for (uint64_t h : edge) { ++n; bad += ct_bucket(h, s) != h % s; }
    for (int i = 0; i < 200000; ++i) { const uint64_t h = g(); ++n; bad += ct_bucket(h, s) != h % s; }
  }
  std::printf("bucket %ld %ld\n", n, bad);
  long rn = 0, rbad = 0, kinds[8] = {0};
  for (int i = 0; i < 400000; ++i) {
    CtFrame f{};
    f.status = 2;
    f.ports_ok = 0;                                  // no ports of its own: ICMP, other protocols
    const uint32_t protos[] = {1, 1, 1, 2, 47, 50, 132};
    f.proto = protos[g() % 7];
    const uint32_t lens[] = {34, 41, 42, 60, 64, 69, 70, 98};
    f.L = lens[g() % 8];
    const uint32_t icmps[] = {0, 8, 3, 11, 13, 14, 17, 18, 5};
    f.icmp = icmps[g() % 9];
    f.src = uint32_t(g());
    f.dst = (g() % 4 == 0) ? f.src : uint32_t(g());  // equal addresses: portRev = ipRev
    f.own = uint32_t(g());
    f.isrc = uint32_t(g()); f.idst = uint32_t(g()); f.iproto = uint32_t(g() % 256);
    f.isport = uint32_t(g() % 65536); f.idport = uint32_t(g() % 65536);
    const uint32_t chain = uint32_t(g() % 4);
    const bool pass = g() % 2, labeled = g() % 5 != 0;
    const int32_t o0 = int32_t(g() % 2000) - 4;
    const uint32_t kb = 8 + uint32_t(g() % 23), sentinel = (1u << kb) - 1;
    uint32_t stale = uint32_t(g());
    if (g() % 4 == 0) stale = (stale & 0xffffu) | (stale & 0xffffu) << 16;   // equal ports
    CtFrame t = f; t.stale = stale;
    CtFrame p = f; p.stale = uint32_t(g());          // whatever the launch had
    const CtWalkOut want = ct_walk_rec(t, chain, pass, labeled, o0, sentinel);
    CtWalkOut got = ct_walk_rec(p, chain, pass, labeled, o0, sentinel);
    if (!labeled || want.kind == kCtKErr) continue;  // (ct_stale_fix marks only labelled records; K_ERR keys on the quote)
    got.key = ct_rec_restale(got.w[0], got.w[1], got.w[2], got.w[6], stale, sentinel);
    ++rn; ++kinds[want.kind & 7];
    bool same = got.key == want.key;
    for (int w = 0; w < 8; ++w) same = same && got.w[w] == want.w[w];
    rbad += !same;
  }
  std::printf("restale %ld %ld kinds %ld %ld %ld %ld %ld %ld %ld %ld\n", rn, rbad, kinds[0], kinds[1], kinds[2],
              kinds[3], kinds[4], kinds[5], kinds[6], kinds[7]);
  return 0;
}
'''


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    d = tmp_path_factory.mktemp("ctrec")
    src, exe = d / "t.cpp", d / "t"
    src.write_text(SRC)
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{ROOT}/polycube_amd/csrc", f"-I{ROOT}/include", str(src), "-o",
                    str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    return {line.split()[0]: [int(x) for x in line.split()[1:] if x.lstrip("-").isdigit()] for line in out if line}


def test_bucket_fold_equals_modulo(results):
    n, bad = results["bucket"]
    assert n > 4_000_000 and bad == 0


def test_restale_completes_the_record(results):
    r = results["restale"]
    n, bad, kinds = r[0], r[1], r[2:]
    assert n > 100_000 and bad == 0
    # labelled frames without ports: echo, echo reply, other ICMP (INVALID), non-ICMP protocols, short drops
    assert kinds[0] and kinds[1] and kinds[4] and kinds[5] and kinds[7], kinds
