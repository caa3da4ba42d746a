"""Drive lists of (key, iv, seq, aad, payload) records through the batch API of libptls_hip.so."""
import numpy as np
import torch

import ptls_hip


def _dev(arr, total):
    buf = np.zeros(max(total, 16) + 16, dtype=np.uint8)
    if arr is not None:
        buf[: len(arr)] = arr
    return torch.from_numpy(buf).cuda()


class HostBatch:
    """records: list of (key, iv, seq, aad, payload).  Each distinct (key, iv) gets its own slot;
    records keep their order (callers group same-key records when they care about speed)."""

    def __init__(self, engine, records, align=16):
        self.engine = engine
        self.records = records
        key_len = len(records[0][0])
        assert all(len(r[0]) == key_len for r in records)
        slots, keys, ivs, slot_of = {}, [], [], []
        for key, iv, *_ in records:
            k = (bytes(key), bytes(iv))
            if k not in slots:
                slots[k] = len(slots)
                keys.append(k[0])
                ivs.append(k[1])
            slot_of.append(slots[k])
        self.keyset = ptls_hip.KeySet(engine, key_len, len(slots))
        self.keyset.set(0, b"".join(keys), b"".join(ivs))
        self.slot_of = slot_of
        self.align = align
        lens = [len(r[4]) for r in records]
        aad_lens = [len(r[3]) for r in records]
        seqs = [r[2] for r in records]
        self.lens = lens
        self.recs, self.in_total, self.out_total, self.aad_total = ptls_hip.layout_records(
            lens, aad_lens, slot_of, seqs, align=align, tag_in_input=True)
        self.aad = np.zeros(self.aad_total, dtype=np.uint8)
        for r, rec in zip(records, self.recs):
            if len(r[3]):
                self.aad[rec["aad_off"]: rec["aad_off"] + len(r[3])] = np.frombuffer(bytes(r[3]), np.uint8)
        self.batch = ptls_hip.Batch(engine, self.recs)

    def close(self):
        self.batch.close()
        self.keyset.close()

    def _input(self, payloads):
        buf = np.zeros(self.in_total, dtype=np.uint8)
        for p, rec in zip(payloads, self.recs):
            if len(p):
                buf[rec["in_off"]: rec["in_off"] + len(p)] = np.frombuffer(bytes(p), np.uint8)
        return buf

    def seal(self, lanes=0, in_place=False, wg=0):
        self.batch.set_lanes(lanes)
        self.batch.set_workgroup(wg)
        d_in = _dev(self._input([r[4] for r in self.records]), self.in_total)
        d_aad = _dev(self.aad, self.aad_total)
        if in_place:  # out_off must then equal in_off: use the input layout for both
            recs = self.recs.copy()
            recs["out_off"] = recs["in_off"]
            b = ptls_hip.Batch(self.engine, recs)
            b.set_lanes(lanes)
            b.seal(self.keyset, d_in, d_aad, d_in)
            torch.cuda.synchronize()
            b.close()
            host = d_in.cpu().numpy()
            return [host[r["in_off"]: r["in_off"] + r["len"] + 16].tobytes() for r in recs]
        d_out = _dev(None, self.out_total)
        self.batch.seal(self.keyset, d_in, d_aad, d_out)
        torch.cuda.synchronize()
        host = d_out.cpu().numpy()
        return [host[r["out_off"]: r["out_off"] + r["len"] + 16].tobytes() for r in self.recs]

    def open(self, sealed, lanes=0, wg=0):
        """sealed: list of ct||tag per record.  Returns (results, plaintexts)."""
        self.batch.set_lanes(lanes)
        self.batch.set_workgroup(wg)
        d_in = _dev(self._input(sealed), self.in_total)
        d_aad = _dev(self.aad, self.aad_total)
        d_out = _dev(None, self.out_total)
        d_res = torch.zeros(len(self.records), dtype=torch.int64, device="cuda")
        self.batch.open(self.keyset, d_in, d_aad, d_out, d_res)
        torch.cuda.synchronize()
        host = d_out.cpu().numpy()
        res = [int(x) & ((1 << 64) - 1) for x in d_res.cpu().numpy().tolist()]
        pts = [host[r["out_off"]: r["out_off"] + r["len"]].tobytes() for r in self.recs]
        return res, pts
