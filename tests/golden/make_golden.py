#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by RUNNING THE REFERENCE ITSELF.

The reference engine is lib/fusion.c compiled unmodified from /root/reference by oracle/Makefile into
oracle/_ref/libptls_fusion_ref.so and reached through picotls's public AEAD API (oracle/ref_harness.c:
ptls_aead_new_direct + ptls_aead_encrypt / ptls_aead_encrypt_s / ptls_aead_xor_iv).

Outputs (data only -- inputs are re-derivable from the documented splitmix64 generator):
  kats.json     the known-answer vectors held by the reference's own t/fusion.c (copied as data) and
                the same vectors re-run through the reference build here.
  sweep.json    length sweep L x AAD x {128,256}: SHA-256 of ct||tag, plus the
                full output for L <= 97.
  configs.json  per-BASELINE-config sample records (first/last 64 and shard seams, §8(c)(iii)):
                SHA-256 of ct||tag per record.
  c4_keyruns.npy  configs[3]'s WHOLE key runs of keys 0..255 (64 records each, 16 384 records, AES-256, mixed
                lengths): SHA-256 of ct||tag per record, uint8[16384][32] in key-run order (key j's records
                i = j + 65536 s, s = 0..63).  The config samples above hold <= 8 records per key, which the planner
                sends to the sparse kernel; these runs take the 32-lane batch kernel the full configs[3] runs.

Run:  make -C oracle && python3 tests/golden/make_golden.py [c4_keyruns]
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle_lib import Oracle, Ref, tls_aad  # noqa: E402

SWEEP_L = list(range(0, 98)) + list(range(1328, 1340)) + [1350, 4095, 4096, 4097, 16383, 16384]
SWEEP_A = [0, 5, 13, 20, 32]
SWEEP_SEED = 0x7377656570000000  # "sweep"

# BASELINE.json configs; n = records, L = payload bytes (None = mixed), keys = #keys
CONFIGS = {
    "c2_tls16k_aes128": dict(n=1 << 20, L=16384, key_len=16, keys=1, aad="tls"),
    "c3_quic1350_aes128": dict(n=4 << 20, L=1350, key_len=16, keys=1, aad="quic"),
    "c4_mixed_aes256_64k": dict(n=4 << 20, L=None, key_len=32, keys=1 << 16, aad="tls"),
    "c5_quic1350_aes128_8gpu": dict(n=32 << 20, L=1350, key_len=16, keys=1, aad="quic"),
}


def sweep_inputs(o, idx, key_len, L, A):
    s = o.stream(SWEEP_SEED ^ idx, key_len + 12 + 8 + A + L)
    key, iv = s[:key_len], s[key_len:key_len + 12]
    seq = int.from_bytes(s[key_len + 12:key_len + 20], "little") >> 8  # keep it < 2^56
    aad = s[key_len + 20:key_len + 20 + A]
    pt = s[key_len + 20 + A:]
    return key, iv, seq, aad, pt


def config_record(o, cfg, i):
    """inputs of record i of a BASELINE config"""
    L = cfg["L"] if cfg["L"] is not None else o.mixed_len(i)
    j = i % cfg["keys"]
    seq = i // cfg["keys"]
    key, iv = o.gen_key(j, cfg["key_len"])
    aad = tls_aad(L) if cfg["aad"] == "tls" else o.gen_quic_aad(i)
    return key, iv, seq, aad, o.gen_record(i, L)


def config_samples(cfg):
    """first / last 64 records of every rank's shard at up to 8 ranks (bench.py: rank r owns records [r n, (r + 1) n)
    of a per-GPU config, weak scaling; configs[4] is one 32M batch in 8 shards of 4M) and both sides of every seam"""
    n = cfg["n"]
    shard = 4 << 20 if n == 32 << 20 else n
    total = n if n == 32 << 20 else 8 * n
    idx = []
    for r in range(total // shard):
        idx += list(range(r * shard, r * shard + 64)) + list(range((r + 1) * shard - 64, (r + 1) * shard))
        if r:
            idx += [r * shard - 1, r * shard]
    return sorted(set(idx))


C4_KEYRUN_KEYS = 256
C4_KEYRUN_LEN = 64  # records per key in configs[3]: 4M records over 64K keys


def c4_keyrun_index():
    """record indices of configs[3]'s key runs 0..C4_KEYRUN_KEYS-1, in key-run order"""
    keys = CONFIGS["c4_mixed_aes256_64k"]["keys"]
    return [j + keys * s for j in range(C4_KEYRUN_KEYS) for s in range(C4_KEYRUN_LEN)]


def make_c4_keyruns(o, r):
    import numpy as np
    cfg = CONFIGS["c4_mixed_aes256_64k"]
    idx = c4_keyrun_index()
    dig = np.zeros((len(idx), 32), dtype=np.uint8)
    for k, i in enumerate(idx):
        out = r.seal(*config_record(o, cfg, i))
        dig[k] = np.frombuffer(hashlib.sha256(out).digest(), np.uint8)
    np.save(os.path.join(HERE, "c4_keyruns.npy"), dig, allow_pickle=False)
    print("c4_keyruns.npy written:", len(idx), "records")


def main():
    o, r = Oracle(), Ref()
    assert Ref.available, "build oracle/_ref first (make -C oracle)"
    if sys.argv[1:] == ["c4_keyruns"]:
        make_c4_keyruns(o, r)
        return
    zero = bytes(16384)

    # ---- KATs from t/fusion.c (data), re-run through the reference build ----
    kats = {"source": "t/fusion.c (reference tests); re-verified against oracle/_ref (lib/fusion.c)"}
    kats["ecb"] = [  # t/fusion.c:76-84
        dict(key=bytes(16).hex(), pt=b"hello world!!!!!".hex(), ct="172afecb50b5f1237814b2f7cb51d0f7"),
        dict(key=bytes(32).hex(), pt=b"hello world!!!!!".hex(), ct="2a033f0627b3554aa4fe5786550736ff"),
    ]
    kats["gfmul"] = dict(  # t/fusion.c:98-226, H in fusion's transformH domain, hash = raw gstate.lo
        H_fusion=b"hello world bye\0".hex(),
        cases=[
            dict(blocks=b"deaddeadbeefbeef".hex(), lo="12d9d9148b3f20bd202aa59e17a8b07b"),
            dict(blocks=b"Lorem ipsum dolor sit amet, con\0".hex(), lo="dadfe89bc78cbd5ca7c1839aa29f8055"),
            dict(blocks=b"The quick brown fox jumps over the lazy dog.".ljust(48, b"\0").hex(),
                 lo="addf91523840f7c385af41b17ded4b56"),
            dict(blocks=b"Lorem ipsum dolor sit amet, consectetur adipiscing elit, sed do eiusmod tempor ".ljust(80, b"\0").hex(),
                 lo="b8ab1ba8f292f389449d39f6b637ca5d"),
            dict(blocks=b"Lorem ipsum dolor sit amet, consectetur adipiscing elit, sed do eiusmod tempor incididunt ut la\0".hex(),
                 lo="52ce2522862c91a4e74ef99a3277bd3e"),
        ])
    hello_pt = b"hello world\n" * 7 + b"\0"  # sizeof(plaintext) incl. NUL = 85
    kats["aead"] = [
        # gcm_basic #1, t/fusion.c:238-247 (ctr = 0 <=> static iv 0, seq 0)
        dict(name="gcm_basic_1", key=bytes(16).hex(), iv=bytes(12).hex(), seq=0, aad=b"hello".hex(), pt=bytes(16).hex(),
             out="0388dace60b6a392f328c2b971b2fe78973fbca65477bf4785b0d561f7e3fd6c"),
        # gcm_basic #2, t/fusion.c:251-273
        dict(name="gcm_basic_2", key=bytes(range(0, 256, 0x11)).hex(), iv=bytes(range(20, 32)).hex(), seq=0,
             aad=bytes(range(20)).hex(), pt=hello_pt.hex(),
             out="d3a81d964c9b02d79ab041074c8ce2e02e83545245cbd468c84345ca91fba37a67ede8d75ee233d13ebf50c24b86835511bb"
                 "174ff578b865eb9a2b8f7708a9601773c507f304c93f674d12a10293c23cd3f85933d501c3bbaae63fbb2366942628"
                 "43a5fd2f"),
        # gcm_capacity, t/fusion.c:278-283
        dict(name="gcm_capacity", key=bytes(16).hex(), iv=bytes(12).hex(), seq=0, aad=b"a".hex(), pt=b"X".hex(),
             out="5b27215ed81a702e3941c80577d52fcb57"),
    ]
    tv = [(13, 17, "1b4e515384e8aa5bb781ee12549a2ccf", "4576f18ef3ae9dfd37cf72c4592da874"),
          (13, 32, "84030586f55adf8ac3c145913c6fd0f8", None), (13, 64, "66165d39739c50c90727e7d49127146b", None),
          (13, 65, "eb3b75e1d4431e1bb67da46f6a1a0edd", None), (13, 79, "8f4a96c7390c26bb15b68865e6a861b9", None),
          (13, 80, "5cc2554857b19e7a9e18d015feac61fd", None), (13, 81, "5a65f0d4db36c981bf7babd11691fe78", None),
          (13, 95, "6a8a51152efe928999a610d8a7b1df9d", None), (13, 96, "6b9c468e24ed96010687f3880a044d42", None),
          (13, 97, "1b4eb785b884a7d4fdebaff81c1c12e8", None), (22, 1328, "0507baaece8d573774c94e8103821316", None),
          (21, 1329, "dd70d59030eadb6313e778046540a253", None), (20, 1330, "f1b456b955afde7603188af0124a32ef", None),
          (13, 1337, "a22deec51250a7eb1f4384dea5f2e890", None), (12, 1338, "42102b0a499b2efa89702ece4b0c5789", None),
          (11, 1339, "9827f0b34252160d0365ffaa9364bedc", None), (0, 80, "98885a3a22bd4742fe7b72172193b163", None),
          (0, 96, "afd649fc51e14f3966e4518ad53b9ddc", None), (20, 85, "afe8b727057c804a0525c2914ef856b0", None)]
    kats["gcm_test_vectors"] = [  # t/fusion.c:309-331: key 0, iv 0, aad/pt all-zero; supp: hp key 01*16, sample at +2
        dict(aadlen=a, ptlen=p, tag=t, supp=s if s is not None else "a062016e90dcc316d061fde5424cf34f")
        for a, p, t, s in tv]
    kats["gcm_iv96"] = dict(  # t/fusion.c:347-377: iv xor'ed with {0,1,2,3} gives gcm_basic_2's iv
        key=bytes(range(0, 256, 0x11)).hex(), iv=bytes([20, 20, 20, 20] + list(range(24, 32))).hex(),
        xor=bytes([0, 1, 2, 3]).hex(), bad_xor=bytes([0x89, 0xab, 0xcd, 0xef]).hex(), expect_same_as="gcm_basic_2")

    # self-check every KAT against the reference build and the oracle before writing anything
    for v in kats["aead"]:
        args = (bytes.fromhex(v["key"]), bytes.fromhex(v["iv"]), v["seq"], bytes.fromhex(v["aad"]),
                bytes.fromhex(v["pt"]))
        assert r.seal(*args).hex() == v["out"] == o.seal(*args).hex(), v["name"]
    for v in kats["gcm_test_vectors"]:
        out, supp = r.seal_supp(bytes(16), bytes(12), 0, zero[:v["aadlen"]], zero[:v["ptlen"]], b"\x01" * 16, 2)
        assert out[v["ptlen"]:].hex() == v["tag"] and supp.hex() == v["supp"], v
        assert o.seal(bytes(16), bytes(12), 0, zero[:v["aadlen"]], zero[:v["ptlen"]]) == out
    iv96 = kats["gcm_iv96"]
    assert r.seal_iv96(bytes.fromhex(iv96["key"]), bytes.fromhex(iv96["iv"]), bytes.fromhex(iv96["xor"]), 0,
                       bytes(range(20)), hello_pt).hex() == kats["aead"][1]["out"]
    for c in kats["gfmul"]["cases"]:
        assert o.fusion_domain_ghash(bytes.fromhex(kats["gfmul"]["H_fusion"]), bytes.fromhex(c["blocks"])).hex() == c["lo"]
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(kats, f, indent=1)

    # ---- length sweep ----
    sweep = dict(source="oracle/_ref (lib/fusion.c via ptls_aead_encrypt)", seed=SWEEP_SEED,
                 derivation="stream(seed ^ idx) = key | iv(12) | seq(8, LE >> 8) | aad(A) | pt(L)", vectors=[])
    idx = 0
    for key_len in (16, 32):
        for L in SWEEP_L:
            for A in SWEEP_A:
                key, iv, seq, aad, pt = sweep_inputs(o, idx, key_len, L, A)
                out = r.seal(key, iv, seq, aad, pt)
                assert r.open(key, iv, seq, aad, out) == (L, pt)
                e = dict(idx=idx, key_len=key_len, L=L, A=A, sha256=hashlib.sha256(out).hexdigest())
                if L <= 97:
                    e["out"] = out.hex()
                sweep["vectors"].append(e)
                idx += 1
    with open(os.path.join(HERE, "sweep.json"), "w") as f:
        json.dump(sweep, f, indent=0)

    # ---- per-config samples ----
    cfgs = dict(source="oracle/_ref (lib/fusion.c via ptls_aead_encrypt)", configs={})
    for name, cfg in CONFIGS.items():
        recs = []
        for i in config_samples(cfg):
            key, iv, seq, aad, pt = config_record(o, cfg, i)
            out = r.seal(key, iv, seq, aad, pt)
            recs.append(dict(i=i, L=len(pt), sha256=hashlib.sha256(out).hexdigest()))
        cfgs["configs"][name] = dict(cfg, records=recs)
    with open(os.path.join(HERE, "configs.json"), "w") as f:
        json.dump(cfgs, f, indent=0)
    print("golden fixtures written:", len(sweep["vectors"]), "sweep vectors")
    make_c4_keyruns(o, r)


if __name__ == "__main__":
    main()
