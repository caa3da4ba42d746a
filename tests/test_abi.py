"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every symbol include/ptls_hip.h
declares, its plugin structs are layout-identical to picotls's, and it fails loudly without a GPU."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

import ptls_hip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ptls_hip.h")
REF_INCLUDE = "/root/reference/include"


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ptls_hip_[a-z0-9_]+)\s*\(", src)))


def declared_data():
    src = open(HEADER).read()
    m = re.findall(r"extern\s+ptls_(?:aead|cipher)_algorithm_t\s+([^;]+);", src)
    return sorted(n.strip() for decl in m for n in decl.split(","))


def test_library_exports_every_declared_symbol():
    L = ptls_hip.lib()
    funcs = declared_functions()
    assert len(funcs) >= 20
    for name in funcs:
        assert hasattr(L, name), name
    for name in declared_data():
        assert ctypes.c_char.in_dll(L, name) is not None, name
    # the Python binding covers exactly what the header declares
    assert sorted(ptls_hip.SIGNATURES) == funcs
    assert sorted(ptls_hip.DATA_SYMBOLS) == declared_data()


def test_record_descriptor_layout():
    assert ptls_hip.RECORD_DTYPE.itemsize == 48
    assert [ptls_hip.RECORD_DTYPE.fields[f][1] for f in ("in_off", "out_off", "aad_off", "seq", "len", "aad_len", "key",
                                                          "flags")] == [0, 8, 16, 24, 32, 36, 40, 44]


def _layout(tmp_path, extra):
    exe = tmp_path / ("abi" + str(len(extra)))
    subprocess.check_call(["gcc", "-std=gnu99", "-w", "-include", "string.h", *extra, "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "abi_layout.c"), "-o", str(exe)])
    return subprocess.check_output([str(exe)]).decode()


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")
def test_plugin_structs_match_picotls_abi(tmp_path):
    ours = _layout(tmp_path, [])
    assert "ptls_aead_context_t size 80" in ours and "ptls_hip_record_t size 48" in ours
    if not os.path.exists(os.path.join(REF_INCLUDE, "picotls.h")):
        pytest.skip("reference picotls.h not present (GPU box)")
    theirs = _layout(tmp_path, ["-I", REF_INCLUDE, "-include", "picotls.h"])
    assert ours == theirs


def test_algorithm_objects_mirror_fusion():
    """field values of ptls_hip_aes{128,256}gcm vs ptls_fusion_aes{128,256}gcm (lib/fusion.c:1231-1256)"""
    L = ptls_hip.lib()

    class Algo(ctypes.Structure):  # include/picotls.h:499-560 (layout checked above)
        _fields_ = [("name", ctypes.c_char_p), ("conf", ctypes.c_uint64), ("integ", ctypes.c_uint64),
                    ("ctr", ctypes.c_void_p), ("ecb", ctypes.c_void_p), ("key_size", ctypes.c_size_t),
                    ("iv_size", ctypes.c_size_t), ("tag_size", ctypes.c_size_t), ("fixed_iv", ctypes.c_size_t),
                    ("record_iv", ctypes.c_size_t), ("bits", ctypes.c_uint8), ("align_bits", ctypes.c_uint8),
                    ("context_size", ctypes.c_size_t), ("setup", ctypes.c_void_p)]

    for name, ks, label in (("ptls_hip_aes128gcm", 16, b"AES128-GCM"), ("ptls_hip_aes256gcm", 32, b"AES256-GCM")):
        a = Algo.in_dll(L, name)
        assert a.name == label and a.key_size == ks and a.iv_size == 12 and a.tag_size == 16
        assert a.conf == 0x2000000 and a.integ == 0x40000000000000
        assert (a.fixed_iv, a.record_iv, a.bits & 1, a.align_bits) == (0, 0, 0, 0)
        assert a.context_size >= 80 and a.setup
    # ptls_non_temporal_aes{128,256}gcm (lib/fusion.c:2154-2179): TLS 1.2 IV split, non_temporal, 64-B alignment
    for name, ks, label in (("ptls_hip_non_temporal_aes128gcm", 16, b"AES128-GCM"),
                            ("ptls_hip_non_temporal_aes256gcm", 32, b"AES256-GCM")):
        a = Algo.in_dll(L, name)
        assert a.name == label and a.key_size == ks and a.iv_size == 12 and a.tag_size == 16
        assert a.conf == 0x2000000 and a.integ == 0x40000000000000
        assert (a.fixed_iv, a.record_iv, a.bits & 1, a.align_bits) == (4, 8, 1, 6)
        assert a.context_size >= 80 and a.setup
    from oracle_lib import REF_SO, Ref
    if Ref.available:  # and field for field against the reference's own objects
        ref = ctypes.CDLL(REF_SO)
        for ours, theirs in (("ptls_hip_aes128gcm", "ptls_fusion_aes128gcm"),
                             ("ptls_hip_aes256gcm", "ptls_fusion_aes256gcm"),
                             ("ptls_hip_non_temporal_aes128gcm", "ptls_non_temporal_aes128gcm"),
                             ("ptls_hip_non_temporal_aes256gcm", "ptls_non_temporal_aes256gcm")):
            a, b = Algo.in_dll(L, ours), Algo.in_dll(ref, theirs)
            fields = ("name", "conf", "integ", "key_size", "iv_size", "tag_size", "fixed_iv", "record_iv",
                      "bits", "align_bits")
            assert [getattr(a, f) for f in fields] == [getattr(b, f) for f in fields], ours
            assert (a.ecb is None) == (b.ecb is None)


def test_ctr_objects_mirror_fusion():
    """ptls_hip_aes{128,256}ctr vs ptls_fusion_aes{128,256}ctr (lib/fusion.c:1219-1230), and the AEAD
    objects advertise them as ctr_cipher like fusion's do"""
    L = ptls_hip.lib()

    class Cipher(ctypes.Structure):  # include/picotls.h:408-415
        _fields_ = [("name", ctypes.c_char_p), ("key_size", ctypes.c_size_t), ("block_size", ctypes.c_size_t),
                    ("iv_size", ctypes.c_size_t), ("context_size", ctypes.c_size_t), ("setup", ctypes.c_void_p)]

    for name, ks, label, aead in (("ptls_hip_aes128ctr", 16, b"AES128-CTR", "ptls_hip_aes128gcm"),
                                  ("ptls_hip_aes256ctr", 32, b"AES256-CTR", "ptls_hip_aes256gcm")):
        c = Cipher.in_dll(L, name)
        assert (c.name, c.key_size, c.block_size, c.iv_size) == (label, ks, 1, 16)
        assert c.context_size >= 32 and c.setup
        ctr_field = ctypes.c_void_p.from_address(ctypes.addressof(ctypes.c_char.in_dll(L, aead)) + 24).value
        assert ctr_field == ctypes.addressof(c)


def _gpu_present():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:  # noqa: BLE001
        return False


@pytest.mark.skipif(_gpu_present(), reason="this checks the no-device error path")
def test_fails_loudly_without_device():
    """no CPU fallback: engine construction errors out, and picotls's own ptls_aead_new_direct returns NULL
    for our algorithm (setup_crypto != 0, lib/picotls.c:6467-6470)"""
    L = ptls_hip.lib()
    assert not ptls_hip.is_supported()  # ptls_fusion_is_supported_by_cpu's counterpart says no
    assert not L.ptls_hip_engine_new(0)
    assert "device" in ptls_hip.last_error().lower()
    with pytest.raises(ptls_hip.HipError):
        ptls_hip.Engine(0)
    with pytest.raises(ptls_hip.HipError):  # the fusion-style low-level context too
        ptls_hip.AesGcm(bytes(16), 64)
    from oracle_lib import REF_SO, Ref
    if Ref.available:
        ref = ctypes.CDLL(REF_SO)
        ref.ptls_aead_new_direct.restype = ctypes.c_void_p
        ref.ptls_aead_new_direct.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        algo = ctypes.addressof(ctypes.c_char.in_dll(L, "ptls_hip_aes128gcm"))
        assert not ref.ptls_aead_new_direct(algo, 1, bytes(16), bytes(12))


def test_iv_only_setup_of_a_fresh_context():
    """setup_crypto(key == NULL) on the context ptls_aead_new_direct just made (lib/picotls.c:6458-6473): fusion
    stores the IV and returns 0 (lib/fusion.c:1188-1191) without touching the vtable; so does ptls_hip_aes*gcm,
    recognising the fresh context by its zeroed `super` (no device needed, none touched).  Ours additionally
    gives it get_iv / set_iv / dispose, so the IV reads back and ptls_aead_free releases it."""
    from oracle_lib import Ref
    if not Ref.available:
        pytest.skip("oracle/_ref not built")
    import plugin_driver
    ref = Ref()
    L = ptls_hip.lib()
    iv = bytes(range(40, 52))
    for bits in (128, 256):
        fus = ref.lib.ref_aead_new_iv_only(ref.algo(f"ptls_fusion_aes{bits}gcm"), 1, iv)
        assert fus, "fusion's IV-only setup returns 0"
        f = plugin_driver.AeadContext.from_address(fus)
        assert not (f.do_encrypt or f.do_decrypt or f.dispose_crypto)
        ref.lib.ref_ctx_free_raw(fus)
        for name in (f"ptls_hip_aes{bits}gcm", f"ptls_hip_non_temporal_aes{bits}gcm"):
            algo = ctypes.addressof(ctypes.c_char.in_dll(L, name))
            for is_enc in (0, 1):
                ctx = ref.lib.ref_aead_new_iv_only(algo, is_enc, iv)
                assert ctx, name
                v = plugin_driver.AeadContext.from_address(ctx)
                assert v.algo == algo and not (v.do_encrypt or v.do_encrypt_v or v.do_decrypt)
                got = ctypes.create_string_buffer(12)
                ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)(v.do_get_iv)(ctx, got)
                assert got.raw == iv
                drv = plugin_driver.PluginDriver()  # the reference's lifecycle functions; no device touched
                drv.xor_iv(ctx, b"\x01\x02")  # the reference's ptls_aead_xor_iv over our get_iv / set_iv
                ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)(v.do_get_iv)(ctx, got)
                assert got.raw == bytes([iv[0] ^ 1, iv[1] ^ 2]) + iv[2:]
                assert ref.lib.ref_aead_setup_iv_only(ctx, is_enc, iv) == 0  # again, now on the IV-only context
                drv.free(ctx)  # ptls_aead_free -> our dispose_crypto


def test_aesecb_api_argument_checks():
    """ptls_hip_aesecb_init rejects what fusion's asserts reject (decryption, key sizes other than 16 / 32,
    lib/fusion.c:859-873) with EINVAL, and, without a device, fails with ENODEV leaving the context empty"""
    L = ptls_hip.lib()
    ctx = ptls_hip.AesEcb.Ctx()
    assert L.ptls_hip_aesecb_init(ctypes.addressof(ctx), 0, bytes(16), 16, 0) == -1
    assert L.ptls_hip_aesecb_init(ctypes.addressof(ctx), 1, bytes(24), 24, 0) == -1
    assert not ctx.state
    if not _gpu_present():
        assert L.ptls_hip_aesecb_init(ctypes.addressof(ctx), 1, bytes(16), 16, 0) == -2
        assert not ctx.state and ctx.rounds == 0
        L.ptls_hip_aesecb_dispose(ctypes.addressof(ctx))  # no-op on an empty context


def test_partition_bytes_matches_bench_rule():
    """ptls_hip_partition_bytes (host-only, the node API's split) == bench.py's partition_bytes on configs[3]'s lengths"""
    import numpy as np
    import sys
    sys.path.insert(0, ROOT)
    import bench
    lens = bench.record_lengths(bench.CONFIGS["c4"], np.arange(20000, dtype=np.uint64))
    recs = np.zeros(len(lens), dtype=ptls_hip.RECORD_DTYPE)
    recs["len"] = lens
    for parts in (1, 2, 3, 7, 8):
        assert ptls_hip.partition_bytes(recs, parts) == bench.partition_bytes(lens, parts)
    assert ptls_hip.partition_bytes(recs[:0], 4) == [0, 0, 0, 0, 0]
    eq = np.zeros(4096, dtype=ptls_hip.RECORD_DTYPE)
    eq["len"] = 1350
    assert ptls_hip.partition_bytes(eq, 4) == [0, 1024, 2048, 3072, 4096]


def test_node_fails_loudly_without_device():
    """the multi-device node has no CPU path either"""
    import torch
    if torch.cuda.is_available():
        pytest.skip("needs a machine without a GPU")
    with pytest.raises(ptls_hip.HipError):
        ptls_hip.Node([0], 16, 1)


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc missing")
@pytest.mark.parametrize("switch", ["DEAL_MUTANT=1", "DEAL_MUTANT=3", "KS_STAMPS=1"])
def test_product_build_refuses_wrong_output_switches(switch, tmp_path):
    """the product objects are compiled with PTLS_HIP_PRODUCT (hsig-picotls_amd/Makefile PROD): a test-mutant switch
    (wrong output by design) or a diagnostic one is then a compile error, not a library"""
    src = os.path.join(ROOT, "hsig-picotls_amd", "csrc", "sparse_kernel.hip")
    inc = ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "hsig-picotls_amd", "csrc")]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only", "-DPTLS_HIP_PRODUCT=1", "-D" + switch,
           *inc, src]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "test-mutant or diagnostic switch" in r.stderr


def test_product_sources_carry_no_experiment_switches():
    """the product sources hold the shipping design only.  Every preprocessor conditional in them is
    an include guard, the x86 host pause, or one of the switches the builds use: the TEST-ONLY dealing mutants
    (DEAL_MUTANT), the diagnostic stamp builds (KS_STAMPS, STAMP_PHASES, WORKER_STAMPS) and the product guard; the
    rejected variants are measured in EXPERIMENTS.md, not kept in the code"""
    import re
    allowed = {"PTLS_HIP_BATCH_KERNEL_H", "PTLS_HIP_INTERNAL_H", "PTLS_HIP_HOST_H", "PTLS_HIP_PLUGIN_H", "PTLS_HIP_GF128_H", "PTLS_HIP_H", "PTLS_HIP_PRODUCT", "DEAL_MUTANT",
               "KS_STAMPS", "STAMP_PHASES", "WORKER_STAMPS", "__x86_64__", "__i386__", "GF128_FN"}
    csrc = os.path.join(ROOT, "hsig-picotls_amd", "csrc")
    seen = set()
    for name in sorted(os.listdir(csrc)):
        with open(os.path.join(csrc, name)) as f:
            for ln in f:
                m = re.match(r"\s*#\s*(if|ifdef|ifndef|elif)\b(.*)", ln)
                if m:
                    seen |= set(re.findall(r"[A-Za-z_][A-Za-z0-9_]*", m.group(2))) - {"defined"}
    assert seen <= allowed, sorted(seen - allowed)
