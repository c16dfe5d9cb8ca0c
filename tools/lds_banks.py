#!/usr/bin/env python3
"""LDS bank-conflict model of the exchanges in K1/K2 (gfx950 rules from
MI355X_MICROARCH.md §LDS): a wave64 LDS instruction is serviced in fixed lane
groups; within a group, each extra distinct dword address on a bank adds one
cycle.

  instruction      lane groups                          bank of dword d
  ds_read_b64      2 x 32 contiguous                    d mod 64
  ds_write_b64     4 x 16 contiguous                    d mod 32
  ds_read_b128     4 x 16 ({0-3,12-15,20-27}, ...)      d mod 64
  ds_write_b128    8 x 8 contiguous                     d mod 32
  ds_read_b32 / ds_write_b32   2 x 32                   d mod 32

usage: lds_banks.py            -> cycles (and the conflict-free minimum) per
                                  wave-instruction of each access pattern
"""
import sys

R128 = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
        [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
R128 = R128 + [[x + 32 for x in g] for g in R128]

GROUPS = {
    "read_b64": ([list(range(0, 32)), list(range(32, 64))], 64, 2),
    "write_b64": ([list(range(i, i + 16)) for i in range(0, 64, 16)], 32, 2),
    "read_b128": (R128, 64, 4),
    "write_b128": ([list(range(i, i + 8)) for i in range(0, 64, 8)], 32, 4),
    "read_b32": ([list(range(0, 32)), list(range(32, 64))], 32, 1),
    # ds_read2_b64 / ds_read2st64_b64: each of the two 8-B accesses in 4 x 16
    # contiguous lane groups, banks mod 32 (MI355X_MICROARCH.md §LDS); model
    # one access per call
    "read2_b64_access": ([list(range(i, i + 16)) for i in range(0, 64, 16)], 32, 2),
    "write_b32": ([list(range(0, 32)), list(range(32, 64))], 32, 1),
}


def cycles(kind, dword_addr):
    """dword_addr[lane] = first dword of the lane's access."""
    groups, nb, width = GROUPS[kind]
    total = 0
    for g in groups:
        banks = {}
        for lane in g:
            for k in range(width):
                d = dword_addr[lane] + k
                banks.setdefault(d % nb, set()).add(d)
        total += max(len(s) for s in banks.values())
    return total, len(groups)


def pad8(i):
    return i + (i >> 3)


def fft_bin(t, j, N):
    C = max(N // 512, 1)
    T = N // 8
    return t + j * T if C == 1 else (t >> 6) + C * ((t & 63) + 64 * j)


def zslot(f, N, P=8):
    """bin-slot layout: bins f = w (mod C) contiguous, regions N/C + P apart"""
    C = max(N // 512, 1)
    return f if C == 1 else (f % C) * (N // C + P) + f // C


def report(name, kind, per_wave):
    """per_wave: list over (wave, j) of the 64 lanes' dword addresses"""
    cyc = mn = 0
    for addrs in per_wave:
        c, m = cycles(kind, addrs)
        cyc += c
        mn += m * (GROUPS[kind][2] * 0 + 1) if False else m
    print(f"{name:58s} {kind:10s} {cyc / len(per_wave):5.2f} cycles/instr (min {mn / len(per_wave):.0f})")


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    T = N // 8
    waves = range(max(T // 64, 1))
    lanes = range(64)
    # K1: bins of fft_dif to LDS, then the split's natural-order reads
    report("K1 scatter lds[pad8(fft_bin)]", "write_b64",
           [[2 * pad8(fft_bin(64 * w + l, j, N)) for l in lanes] for w in waves for j in range(8)])
    report("K1 split read lds[pad8(f)], f = t + jT", "read_b64",
           [[2 * pad8(64 * w + l + j * T) for l in lanes] for w in waves for j in range(4)])
    report("K1 split read lds[pad8(N - f)]", "read_b64",
           [[2 * pad8((N - (64 * w + l + j * T)) % N) for l in lanes] for w in waves for j in range(4)])
    report("slot layout: scatter lds[zslot(fft_bin)]", "write_b64",
           [[2 * zslot(fft_bin(64 * w + l, j, N), N) for l in lanes] for w in waves for j in range(8)])
    report("slot layout: read lds[zslot(f)]", "read_b64",
           [[2 * zslot(64 * w + l + j * T, N) for l in lanes] for w in waves for j in range(4)])
    report("slot layout: read lds[zslot(N - f)]", "read_b64",
           [[2 * zslot((N - (64 * w + l + j * T)) % N, N) for l in lanes] for w in waves for j in range(4)])
    GPW = 2
    report("K1 staging stg[(t + jT) GPW + grp] (float4)", "write_b128",
           [[4 * ((64 * w + l + j * T) * GPW + 0) for l in lanes] for w in waves for j in range(4)])
    # K2 packed group: partner reads of Z(N - fy) in the bin layout
    report("K2 packed: read lds[pad8(N - fft_bin)]", "read_b64",
           [[2 * pad8((N - fft_bin(64 * w + l, j, N)) % N) for l in lanes] for w in waves for j in range(8)])
    report("slot layout: read lds[zslot(N - fft_bin)]", "read_b64",
           [[2 * zslot((N - fft_bin(64 * w + l, j, N)) % N, N) for l in lanes] for w in waves for j in range(8)])
    # K2 op table (float2 per bin entry): natural index vs k2_tix
    C = max(N // 512, 1)
    Q = (N // 2 + 1 + C - 1) // C

    def tix(e):
        return e if C == 1 else (e % C) * Q + e // C
    ent = lambda t, j: fft_bin(t, j, N) if j < 4 else N - fft_bin(t, j, N)
    report("K2 op table tab0[natural entry]", "read_b64",
           [[2 * ent(64 * w + l, j) for l in lanes] for w in waves for j in range(8)])
    report("K2 op table tab0[k2_tix(entry)]", "read_b64",
           [[2 * tix(ent(64 * w + l, j)) for l in lanes] for w in waves for j in range(8)])
    # K2 Q staging: stg[((k/TK) GPW) TK + k%TK + TK grp], k = t + jT - rb (TK = 2)
    TK, rb = 2, 482
    report("K2 Q staging write (c2), group 0", "write_b64",
           [[2 * ((((64 * w + l + j * T - rb) % N) // TK) * GPW * TK + ((64 * w + l + j * T - rb) % N) % TK)
             for l in lanes] for w in waves for j in range(8)])
    # round 4: canvas-row staging slot s0 = ((t >> 1) GPW + grp) TK + (t & 1),
    # swizzled c2 slot i ^ (((i >> 4) & 1) << 1); reads float4 r ^ ((r >> 3) & 1)
    swz = lambda i: i ^ (((i >> 4) & 1) << 1)
    swz4 = lambda r: r ^ ((r >> 3) & 1)
    for g_ in (0, 1):
        s0 = lambda t: (((t >> 1) * GPW + g_) * TK + (t & 1))
        report(f"K2 Q staging write linear, group {g_}", "write_b64",
               [[2 * (s0(64 * w + l) + j * (T // 2) * GPW * TK) for l in lanes] for w in waves for j in range(8)])
        report(f"K2 Q staging write swizzled, group {g_}", "write_b64",
               [[2 * (swz(s0(64 * w + l)) + j * (T // 2) * GPW * TK) for l in lanes] for w in waves for j in range(8)])
    for off in (0, 482):
        report(f"K2 Q staging read float4 linear (+{off})", "read_b128",
               [[4 * (64 * w + l + off) for l in lanes] for w in range(GPW * T // 64)])
        report(f"K2 Q staging read float4 swizzled (+{off})", "read_b128",
               [[4 * swz4(64 * w + l + off) for l in lanes] for w in range(GPW * T // 64)])

    # k_sb_cols staging at R = 2, GPW = 2 (1080p Hn = 1084; the read pattern
    # repeats every 32 row groups): row-group-major vs column-major at stride S
    rb, Hn = 482, 1084
    S = (Hn + 1) // 2 * 2
    S = (S + 15) // 32 * 32 + 16
    kk = lambda t, j: (t + j * T - rb) % N
    for g_ in (0, 1):
        report(f"sb_stg write row-group-major, column {g_}", "write_b64",
               [[2 * ((kk(64 * w + l, j) // 2) * 4 + 2 * g_ + kk(64 * w + l, j) % 2) for l in lanes]
                for w in waves for j in range(8)])
        report(f"sb_stg write column-major S = {S}, column {g_}", "write_b64",
               [[2 * (g_ * S + kk(64 * w + l, j)) for l in lanes] for w in waves for j in range(8)])
    report("sb_stg read float4 row-group-major", "read_b128", [[4 * (64 * w + l) for l in lanes] for w in range(8)])
    report(f"sb_stg read float4 column-major S = {S}", "read_b128",
           [[2 * ((e % 2) * S + 2 * (e // 2)) for e in (64 * w + l for l in lanes)] for w in range(8)])


if __name__ == "__main__":
    main()


# ---- Stockham passes of fft_regs / fft_pass (mm_fft.hpp) -------------------
def passes(log2n):
    out, ns = [], 1
    full = log2n // 3
    for p in range((log2n + 2) // 3):
        r = 8 if p < full else (4 if log2n % 3 == 2 else 2)
        out.append((r, ns))
        ns *= r
    return out


def xpad(i, log2n, ns):
    if log2n < 9 or ns == 1:
        s, a = 3, 1
    elif ns == 8:
        s, a = 5, 4
    else:
        s, a = 30, 0
    return i + a * (i >> s)


def stockham_report(tag, log2n, T, waves):
    """every exchange of the transform over T threads (lane l of wave w:
    t = 64 w + l): writes y[(b/Ns) Ns R + b%Ns + m Ns], reads x[t + j T]"""
    N = 1 << log2n
    ps = passes(log2n)
    for p, (r, ns) in enumerate(ps[:-1]):
        B = 8 // r
        wr = []
        for w in waves:
            for q in range(B):
                for m in range(r):
                    addrs = []
                    for l in range(64):
                        t = 64 * w + l
                        b = t + q * T
                        idx = (b // ns) * ns * r + b % ns + m * ns
                        addrs.append(2 * xpad(idx, log2n, ns))
                    wr.append(addrs)
        report(f"{tag} pass {p} (R{r} Ns{ns}) write", "write_b64", wr)
        rd = [[2 * xpad(64 * w + l + j * T, log2n, ns) for l in range(64)] for w in waves for j in range(8)]
        report(f"{tag} pass {p} (R{r} Ns{ns}) read", "read_b64", rd)


def k34_report(N=2048, x0=64):
    T = N // 8
    waves = range(T // 64)
    stockham_report("K34/K3 fft_regs", N.bit_length() - 1, T, waves)
    # |z| rows: raw[t + jT], raw[N + t + jT] (floats)
    report("K34 |z| write raw[t + jT]", "write_b32", [[64 * w + l + j * T for l in range(64)] for w in waves for j in range(8)])
    # horizontal blur, round 3 code: the compiler read taps c-2 .. c+5 (c = x0 +
    # 4q) as two ds_read2_b64 of 16 B at 8-B aligned c-2 and c+2 (two accesses
    # each): 2-way conflicts on every access
    for c0 in (-2, 0, 2, 4):
        report(f"K34 blur (r3) read2_b64 access at c{c0:+d}", "read2_b64_access",
               [[x0 + 4 * (64 * w + l) + c0 for l in range(64)] for w in range(2 * T // 64)])
    # round 4: |z| rows kZShift = 2 floats in, taps c-2 .. c+5 = two aligned ds_read_b128
    for k in (0, 1):
        report(f"K34 blur (r4, zshift) read_b128 #{k}", "read_b128",
               [[x0 + 4 * (64 * w + l) + 4 * k for l in range(64)] for w in range(2 * T // 64)])


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "k34":
    k34_report(int(sys.argv[1]))


def xpad(i, ns):
    """mm_fft.hpp xpad for the wave-local 512-point inner transform (LOG2N 9)."""
    s, a = (3, 1) if ns == 1 else ((5, 4) if ns == 8 else (30, 0))
    return i + a * (i >> s)


def fft_wl_report(N=2048):
    """The wave-local transform's LDS traffic per wave (fft_dif / fft_dit at
    C = N / 512 waves, mm_fft.hpp): the cross-wave exchange, then the inner
    512-point Stockham passes' two wave-local exchanges (radix 8; pass 0 at
    Ns = 1 with pad8, pass 1 at Ns = 8 with xpad A = 4, S = 5).  Every K2 / K1
    / K34 transform runs these, so their sum is the FFT share of a kernel's
    LDS cycles (tools/lds_banks.py main() covers the tables and staging)."""
    C = max(N // 512, 1)
    RS = 512 + 64
    lanes = range(64)
    tot = {}

    def rep(name, kind, pats):
        c = [cycles(kind, [2 * e for e in p]) for p in pats]
        got, mn = sum(x[0] for x in c), sum(x[1] for x in c) * (GROUPS[kind][2] if kind != "read_b64" else 1)
        # minimum: each lane group needs width dwords per lane over its banks
        groups, nb, width = GROUPS[kind]
        mn = sum(max(1, len(g) * width // nb) for g in groups) * len(pats)
        tot[name] = (got, mn)
        print(f"{name:58s} {kind:10s} {got / len(pats):5.2f} cycles/instr (min {mn / len(pats):.0f})")

    if C > 1:
        H = 8 // C
        rep("fft_dif cross-wave write lds[m RS + n2]", "write_b64",
            [[m * RS + (l + 64 * C * h) for l in lanes] for h in range(H) for m in range(C)])
        rep("fft_dif cross-wave read reg[l + 64 j]", "read_b64", [[l + 64 * j for l in lanes] for j in range(8)])
    for p_, ns in ((0, 1), (1, 8)):
        rep(f"inner pass {p_} write (Ns = {ns})", "write_b64",
            [[xpad((l // ns) * ns * 8 + l % ns + m * ns, ns) for l in lanes] for m in range(8)])
        rep(f"inner pass {p_} read (Ns = {ns})", "read_b64",
            [[xpad(l + 64 * j, ns) for l in lanes] for j in range(8)])
    got = sum(v[0] for v in tot.values())
    mn = sum(v[1] for v in tot.values())
    print(f"{'one wave-local transform: LDS cycles / conflict-free minimum':58s} {got} / {mn} = {got / mn:.3f}")


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "fft":
    fft_wl_report(int(sys.argv[1]))
