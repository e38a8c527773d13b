"""Randomised SoA logs for differential tests (engine vs C oracle).

Unlike the bench generator (agn_gen_*), these exercise every corner the
reference's semantics has: ragged and empty keys, sparse clocks (DCs missing
from op clocks, from the read snapshot and from SCT), warm reads (SCT set),
reading-transaction matches (TxId == op.txid), invalid effects, keys whose
ops have another type, multi-entry ops and base states.
"""
from __future__ import annotations

import numpy as np

from antidote_amd import _abi
from antidote_amd.encode import EncodedLog, EncodedRead, n_words, state_capacity


def _mask_rows(rng, n, D, p_absent):
    W = n_words(D)
    m = np.zeros((n, W), np.uint64)
    present = rng.random((n, D)) >= p_absent
    for d in range(D):
        m[:, d >> 6] |= present[:, d].astype(np.uint64) << np.uint64(d & 63)
    return m, present


def random_case(seed, crdt, K, D, nmax, *, sparse=False, warm=0.0, txid=0.0, invalid=0.0,
                corrupt=0.0, multi=0.0, base=0.0, n_elems=6, empty=0.1, identity=True):
    rng = np.random.default_rng(seed)
    W = n_words(D)
    lens = rng.integers(0, nmax + 1, K)
    lens[rng.random(K) < empty] = 0
    key_off = np.zeros(K + 1, np.uint64)
    key_off[1:] = np.cumsum(lens)
    E = int(key_off[-1])
    base_t = 1_000_000
    # op clocks: per key a random walk so that reads include a prefix-ish subset
    oc = np.zeros((E, D), np.uint64)
    op_id = np.zeros(E, np.uint32)
    txids = np.zeros(E, np.uint64)
    R = np.zeros((K, D), np.uint64)
    sct = np.zeros((K, D), np.uint64)
    sct_ign = np.ones(K, np.uint8)
    rtx = np.zeros(K, np.uint64)
    for k in range(K):
        a, b = int(key_off[k]), int(key_off[k + 1])
        clk = base_t + rng.integers(0, 50, D)
        ids = np.sort(rng.choice(np.arange(1, 4 * (b - a) + 2), b - a, replace=False)) \
            if b > a else []
        snaps = []
        for j, e in enumerate(range(a, b)):
            c = rng.integers(0, D)
            clk = clk.copy()
            clk[c] += rng.integers(1, 20)
            row = clk - rng.integers(0, 30, D)
            row[c] = clk[c]
            oc[e] = row
            op_id[e] = ids[j]
            txids[e] = rng.integers(1, 6)
            snaps.append(row)
        cut = rng.integers(0, (b - a) + 1)
        Rk = (np.max(np.array(snaps[:cut]), axis=0) if cut else clk - 10) + rng.integers(-4, 16, D)
        R[k] = np.maximum(Rk, 1)
        if rng.random() < warm:
            c2 = rng.integers(0, cut + 1)
            sct[k] = (np.max(np.array(snaps[:c2]), axis=0) if c2 else clk - 40) + \
                rng.integers(-5, 6, D)
            sct_ign[k] = 0
        if rng.random() < txid:
            rtx[k] = rng.integers(1, 6)
    # multi-entry ops: copy the previous entry's id/clock/txid
    if multi and E:
        for k in range(K):
            a, b = int(key_off[k]), int(key_off[k + 1])
            for e in range(a + 1, b):
                if rng.random() < multi:
                    op_id[e], oc[e], txids[e] = op_id[e - 1], oc[e - 1], txids[e - 1]
    log = EncodedLog(crdt_type=crdt, n_dcs=D, key_off=key_off,
                     key_type=np.full(K, crdt, np.uint8), oc=oc, oc_mask=None, op_id=op_id,
                     txid=txids)
    log.key_type[rng.random(K) < corrupt] = _abi.TYPE_MIXED
    if sparse:
        log.oc_mask, present = _mask_rows(rng, E, D, 0.25)
        # the commit DC (max entry) is always present in OpSSCommit
        for e in range(E):
            d = int(np.argmax(oc[e]))
            log.oc_mask[e, d >> 6] |= np.uint64(1 << (d & 63))
        # multi-entry ops share the mask too
        for k in range(K):
            a, b = int(key_off[k]), int(key_off[k + 1])
            for e in range(a + 1, b):
                if op_id[e] == op_id[e - 1]:
                    log.oc_mask[e] = log.oc_mask[e - 1]
    if crdt == _abi.COUNTER_PN:
        eff = rng.integers(-1000, 1001, E).astype(np.int64)
        eff[rng.random(E) < invalid] = _abi.EFFECT_INVALID
        log.eff = eff
    else:
        tag = rng.integers(0, n_elems, E).astype(np.uint32)
        add = np.zeros(E, np.uint64)
        rem_off = np.zeros(E + 1, np.uint32)
        rem = []
        tok_ctr = 1
        for k in range(K):
            a, b = int(key_off[k]), int(key_off[k + 1])
            live: dict = {}
            allt = []
            for e in range(a, b):
                t = int(tag[e])
                if crdt == _abi.REGISTER_MV and rng.random() < 0.1:
                    tag[e] = 0
                    add[e] = 0
                    obs = [x for v in live.values() for x in v]
                    live = {}
                elif rng.random() < 0.7:
                    tok = (k << 24) | tok_ctr
                    tok_ctr += 1
                    add[e] = tok
                    key = t if crdt == _abi.SET_AW else 0
                    cur = live.get(key, [])
                    if rng.random() < 0.25:
                        obs = []
                        live[key] = cur + [tok]
                    else:
                        obs = list(cur)
                        live[key] = [tok]
                    allt.append(tok)
                else:
                    key = t if crdt == _abi.SET_AW else 0
                    obs = list(live.get(key, []))
                    live[key] = []
                # stale / foreign tokens in removal lists (must be no-ops or order-aware)
                if allt and rng.random() < 0.2:
                    obs = obs + [int(rng.choice(allt))]
                rem.extend(obs)
                rem_off[e + 1] = len(rem)
            tok_ctr += 0
        tag[rng.random(E) < invalid] = _abi.TAG_INVALID
        log.tag, log.add_tok, log.rem_off = tag, add, rem_off
        log.rem_tok = np.array(rem if rem else [0], np.uint64)
    Rm = Sm = None
    if sparse:
        Rm, _ = _mask_rows(rng, K, D, 0.03)
        Sm, _ = _mask_rows(rng, K, D, 0.2)
    else:
        Rm = np.zeros((K, W), np.uint64)
        Sm = np.zeros((K, W), np.uint64)
    boff = np.zeros(K + 1, np.uint64)
    btag, btok = [], []
    if crdt != _abi.COUNTER_PN:
        for k in range(K):
            if rng.random() < base:
                pairs = [(int(rng.integers(0, n_elems)), (1 << 60) | (k << 8) | (x + 1))
                         for x in range(int(rng.integers(1, 5)))]
                # the reference's states are ordered: set_aw orddict by elem (tokens in
                # list order), register_mv sorted by {Value, Token}
                pairs.sort(key=(lambda p: p[0]) if crdt == _abi.SET_AW else None)
                for t, tk in pairs:
                    btag.append(t)
                    btok.append(tk)
            boff[k + 1] = len(btag)
    keys = np.arange(K, dtype=np.uint64)
    if not identity:
        keys = rng.permutation(K).astype(np.uint64)
        R, Rm, sct, Sm, sct_ign, rtx = R[keys], Rm[keys], sct[keys], Sm[keys], sct_ign[keys], \
            rtx[keys]
    req = EncodedRead(n_dcs=D, req_type=crdt, keys=keys, R=np.ascontiguousarray(R),
                      R_mask=np.ascontiguousarray(Rm), sct=np.ascontiguousarray(sct),
                      sct_mask=np.ascontiguousarray(Sm), sct_ignore=sct_ign, txid=rtx,
                      base_value=rng.integers(-50, 50, K).astype(np.int64), base_off=boff,
                      base_tag=np.array(btag, np.uint32), base_tok=np.array(btok, np.uint64))
    cap = state_capacity(log, req) if crdt != _abi.COUNTER_PN else None
    return log, req, cap


def compare(crdt, D, a, b, sparse, n):
    """Field-by-field bit-exact comparison of two ResultArrays; returns a list
    of mismatching request indices (empty = identical)."""
    bad = []
    for i in range(n):
        fa, fb = int(a.flags[i]), int(b.flags[i])
        if fa != fb:
            bad.append((i, "flags", fa, fb))
            continue
        if fa & (_abi.F_ERR_CORRUPTED | _abi.F_ERR_UNEXPECTED):
            if int(a.err_pos[i]) != int(b.err_pos[i]):
                bad.append((i, "err_pos", int(a.err_pos[i]), int(b.err_pos[i])))
            continue
        if int(a.hole[i]) != int(b.hole[i]):
            bad.append((i, "hole", int(a.hole[i]), int(b.hole[i])))
        if int(a.count[i]) != int(b.count[i]):
            bad.append((i, "count", int(a.count[i]), int(b.count[i])))
        if not (fa & _abi.F_CT_IGNORE):
            if sparse:
                if not np.array_equal(a.lastct_mask[i], b.lastct_mask[i]):
                    bad.append((i, "lastct_mask"))
                m = [(int(a.lastct_mask[i][d >> 6]) >> (d & 63)) & 1 for d in range(D)]
                va = [int(x) for x, keep in zip(a.lastct[i], m) if keep]
                vb = [int(x) for x, keep in zip(b.lastct[i], m) if keep]
                if va != vb:
                    bad.append((i, "lastct"))
            elif not np.array_equal(a.lastct[i], b.lastct[i]):
                bad.append((i, "lastct"))
        if crdt == _abi.COUNTER_PN:
            if int(a.value[i]) != int(b.value[i]):
                bad.append((i, "value", int(a.value[i]), int(b.value[i])))
        elif not (fa & _abi.F_ERR_CAPACITY):
            if int(a.out_n[i]) != int(b.out_n[i]):
                bad.append((i, "out_n", int(a.out_n[i]), int(b.out_n[i])))
                continue
            o, k = int(a.out_off[i]), int(a.out_n[i])
            if not (np.array_equal(a.out_tag[o:o + k], b.out_tag[o:o + k]) and
                    np.array_equal(a.out_tok[o:o + k], b.out_tok[o:o + k])):
                bad.append((i, "state"))
    return bad
