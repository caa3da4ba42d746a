"""Register-budget guards read from the built gfx950 code objects (hsig-picotls_amd/build/*.o, no GPU needed): the kernel
descriptors' private segment (scratch) sizes.
  - plugin_worker_kernel: none.  A resident kernel with scratch is the first suspect of the one GPU fault of round 3
    (EXPERIMENTS.md E3: constant-space key pointers), and the worker must not touch memory it does not own.
  - the single-record launch (aesgcm_sparse_kernel, 256 threads): none (the plugin's latency path).
  - the sparse batch kernel (768 threads): at most 16 bytes per lane.  Scratch that lives across its record loop is
    evicted to HBM by the streaming records (c4s: 84 B per lane cost +4.9 KB of HBM traffic per record in round 3; round 4's
    32 B were a hoisted lane index and a zero vector reloaded per record, 0.07x of c4s's traffic).
  - the batch kernel (every lanes-per-record value, both workgroup sizes): none (round 4: the table build's hoisted thread
    addresses were reloaded from scratch after every key switch's barrier)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "hsig-picotls_amd", "build")
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernels(obj, tmp_path):
    """{kernel symbol: private_segment_fixed_size} of the gfx950 code object bundled into a host object"""
    fat, co = tmp_path / "fat.bin", tmp_path / "k.co"
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, str(fat)], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True, capture_output=True, text=True).stdout
    out, name = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
        m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", line)
        if m and name is not None:
            out[name] = int(m.group(1))
    return out


@pytest.mark.skipif(not os.path.exists(os.path.join(BUILD, "sparse_kernel.o")) or not os.path.exists(f"{LLVM}/clang-offload-bundler"),
                    reason="needs the in-tree build (__graft_entry__.build()) and the ROCm LLVM tools")
def test_sparse_kernel_scratch_budget(tmp_path):
    ks = _kernels(os.path.join(BUILD, "sparse_kernel.o"), tmp_path)
    worker = [k for k in ks if "plugin_worker_kernel" in k]
    single = [k for k in ks if "aesgcm_sparse_kernel" in k and k.split("EEEv")[0].endswith("Li256")]
    batch = [k for k in ks if "aesgcm_sparse_kernel" in k and k.split("EEEv")[0].endswith("Li768")]
    assert len(worker) == 1 and len(single) == 8 and len(batch) == 8, sorted(ks)
    assert ks[worker[0]] == 0, ("the resident plugin worker uses scratch", ks[worker[0]])
    assert all(ks[k] == 0 for k in single), {k: ks[k] for k in single}
    assert all(ks[k] <= 16 for k in batch), {k: ks[k] for k in batch}


@pytest.mark.skipif(not os.path.exists(os.path.join(BUILD, "batch_g8.o")) or not os.path.exists(f"{LLVM}/clang-offload-bundler"),
                    reason="needs the in-tree build (__graft_entry__.build()) and the ROCm LLVM tools")
@pytest.mark.parametrize("g", [1, 2, 4, 8, 16, 32])
def test_batch_kernel_has_no_scratch(tmp_path, g):
    ks = _kernels(os.path.join(BUILD, f"batch_g{g}.o"), tmp_path)
    batch = [k for k in ks if "aesgcm_batch_kernel" in k]
    assert len(batch) == 16, sorted(ks)  # 2 key sizes x seal / open x aligned / not x 512 / 768 threads
    assert all(ks[k] == 0 for k in batch), {k: ks[k] for k in batch if ks[k]}
