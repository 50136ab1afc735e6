"""LDS bank-conflict model of the fused Swin stage-1 kernels' access patterns (swin.hip
swin_attn96_kernel) for candidate row pitches, from MI355X_MICROARCH.md's per-instruction lane
groups: ds_read_b128 4 x 16 lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59},
{36-43,48-51,60-63}, bank (a/4) mod 64; ds_read_b64(_tr_b16) 2 x 32, mod 64; ds_write_b64 4 x 16
contiguous, mod 32; ds_write_b128 8 x 8 contiguous, mod 32. Cycles of a group = the most distinct
dword addresses on one bank (identical addresses broadcast); extra = cycles - ideal.
    python scripts/probe/lds_conflicts.py

Measured (round 4, Swin-T bs256 kernel trace, 3 alternating pairs): swin_mlp96_kernel's weight
reads, W1 / W2 pitches 208 / 784 -> 224 / 800 (model: 48 -> 0 extra cycles per pattern set):
264 -> 255 us per launch, adopted. swin_attn96_kernel, qkv pitch 592 -> 608 (model: fewer
conflicts): 271 -> 284 us, proj pitch 208 -> 224: 271 -> 272 us - the model does not capture
what bounds that kernel's qkv traffic (the transposed V reads are the least certain lane-group
assumption); both kept at 592 / 208."""
import itertools

G128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G128 += [[l + 32 for l in g] for g in G128]
GROUPS = {"r128": (G128, 64, 4), "r64": ([list(range(32)), list(range(32, 64))], 64, 2),
          "w64": ([list(range(16 * i, 16 * i + 16)) for i in range(4)], 32, 2),
          "w128": ([list(range(8 * i, 8 * i + 8)) for i in range(8)], 32, 4)}


def cycles(kind, addr):  # addr: lane -> byte address
    groups, nb, nd = GROUPS[kind]
    tot = 0
    for g in groups:
        banks = {}
        for l in g:
            for d in range(nd):
                w = addr(l) // 4 + d
                banks.setdefault(w % nb, set()).add(w)
        tot += max(len(v) for v in banks.values())
    return tot


def ideal(kind):
    groups, nb, nd = GROUPS[kind]
    return sum(max(1, (len(g) * nd + nb - 1) // nb) for g in groups)


def patterns(ROW, QROW):
    c16 = lambda l: l & 15  # noqa: E731
    g = lambda l: l >> 4  # noqa: E731
    P = []
    for tt, ks in itertools.product(range(4), range(3)):  # P1 bx reads
        P.append(("P1 bx", "r128", lambda l, tt=tt, ks=ks: (16 * tt + c16(l)) * ROW + 64 * ks + 16 * g(l)))
    for tt, ft in itertools.product(range(4), range(5)):  # P1 qkv writes
        P.append(("P1 qkv w", "w64", lambda l, tt=tt, ft=ft: (16 * tt + c16(l)) * QROW + (16 * ft + 4 * g(l)) * 2))
    for qt, h in itertools.product(range(4), range(3)):
        P.append(("P2 q", "r128", lambda l, qt=qt, h=h: (16 * qt + c16(l)) * QROW + (32 * h + 8 * g(l)) * 2))
        for kt in range(4):
            P.append(("P2 k", "r128", lambda l, kt=kt, h=h: (16 * kt + c16(l)) * QROW + (96 + 32 * h + 8 * g(l)) * 2))
        for ks, dt, half in itertools.product(range(2), range(2), range(2)):
            P.append(("P2 v tr", "r64", lambda l, ks=ks, dt=dt, h=h, half=half:
                      (ks * 32 + 4 * g(l) + ((l >> 2) & 3) + 16 * half) * QROW + (192 + 32 * h + 16 * dt + 4 * (l & 3)) * 2))
        for dt in range(2):
            P.append(("P2 o w", "w64", lambda l, qt=qt, h=h, dt=dt: (16 * qt + c16(l)) * ROW + (32 * h + 16 * dt + 4 * g(l)) * 2))
    for qt, ks in itertools.product(range(4), range(3)):
        P.append(("P3 bo", "r128", lambda l, qt=qt, ks=ks: (16 * qt + c16(l)) * ROW + 64 * ks + 16 * g(l)))
        for f in range(6):
            P.append(("P3 wp", "r128", lambda l, f=f, ks=ks: (16 * f + c16(l)) * ROW + 64 * ks + 16 * g(l)))
    for qt, f in itertools.product(range(4), range(6)):
        P.append(("P3 xm w", "w64", lambda l, qt=qt, f=f: (16 * qt + c16(l)) * ROW + (16 * f + 4 * g(l)) * 2))
    return P


def mlp_patterns(W1, W2):
    """swin_mlp96_kernel weight fragment reads (ds_read_b128): W1 row hc*32 + ht*16 + c16,
    16-B piece 4*ks + g; W2 row ct*16 + c16, 16-B piece 4*hc + g."""
    c16 = lambda l: l & 15  # noqa: E731
    g = lambda l: l >> 4  # noqa: E731
    P = [("w1", "r128", lambda l, ks=ks: c16(l) * W1 + 64 * ks + 16 * g(l)) for ks in range(3)]
    P += [("w2", "r128", lambda l, hc=hc: c16(l) * W2 + 64 * hc + 16 * g(l)) for hc in range(12)]
    return P


def main():
    for W1, W2 in [(208, 784), (224, 800)]:
        per = {}
        for name, kind, a in mlp_patterns(W1, W2):
            per[name] = per.get(name, 0) + cycles(kind, a) - ideal(kind)
        print(f"MLP W1 {W1} W2 {W2}: extra", per)
    for ROW, QROW in [(208, 592), (200, 592), (216, 592), (208, 600), (208, 608), (200, 600),
                      (216, 600), (208, 584), (200, 584), (216, 608), (224, 592), (208, 624)]:
        per, tot, ext = {}, 0, 0
        for name, kind, a in patterns(ROW, QROW):
            c = cycles(kind, a)
            per[name] = per.get(name, 0) + c - ideal(kind)
            tot += c
            ext += c - ideal(kind)
        print(f"ROW {ROW} QROW {QROW}: cycles {tot} extra {ext}  ", {k: v for k, v in per.items() if v})


if __name__ == "__main__":
    main()
