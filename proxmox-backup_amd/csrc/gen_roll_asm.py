"""Generate roll128_asm.h: hand-scheduled gfx950 bodies of the rolling hash loop used
by scan_main_kernel (DESIGN.md "Kernel: scan_main").

Per byte i of the lane's block:
    addr  = v_perm_b32(d[i/4], lanebase, sel[i%4])     # b*256 + lane*4 (replicated table)
    R[e]  = ds_read_b32(addr)                          # T'[b], issued P bytes ahead
    H     = v_alignbit_b32(H, H, 31)                   # rotl 1
    H     = v_bitop3_b32(H, R[l], R[e], 0x96)          # ^ T'[leave] ^ T'[enter]
    acc   = v_max3_u32(acc, H_even, H_odd)             # every second byte
The ring R[0..127] keeps T' of the previous 128 bytes; the "leave" value of byte i
is R[(i+64) % 128], so no register moves are needed, and a read into R[i] (i >= 64)
is issued only after R[i] was consumed as a leave value (P < 64).  LDS reads return
in order, so one counted s_waitcnt lgkmcnt(n) per group of G bytes retires exactly
the reads that group needs while the next ones stay in flight (lgkmcnt <= 15).

Measured on MI355X (scripts/microbench): a wave64 VOP3 op costs ~4 SIMD cycles in
this mix, so the loop is VALU-bound at ~3.5 VALU/byte; every instruction saved here
is throughput.

    python gen_roll_asm.py > roll128_asm.h
"""
import sys

NA = 4  # rotating address temporaries


def body(nbytes, enter, leave, G, P, acc_init):
    """enter(i)/leave(i): operand index of the ring slot receiving byte i / holding the
    byte 64 positions earlier.  Operands: R 0..127, H1 128, ACC 129, H0 130,
    A 131..131+NA-1, D from 131+NA, then LB and the 4 selector SGPRs."""
    nd = nbytes // 4
    H1, ACC, H0 = "%128", "%129", "%130"
    A = lambda k: f"%{131 + k}"
    D = lambda w: f"%{131 + NA + w}"
    LB = f"%{131 + NA + nd}"
    S = lambda k: f"%{131 + NA + nd + 1 + k}"
    assert P + G <= 15 and G in (2, 4) and P % G == 0
    lines = ["s_waitcnt lgkmcnt(0)"]  # no foreign LGKM op in flight (counted waits below)

    def issue(bs):
        bs = [b for b in bs if b < nbytes]
        for b in bs:  # perms first: no ds_read right behind the VALU op that made its address
            lines.append(f"v_perm_b32 {A(b % NA)}, {D(b // 4)}, {LB}, {S(b % 4)}")
        for b in bs:
            lines.append(f"ds_read_b32 %{enter(b)}, {A(b % NA)}")
        return bs

    for b in range(0, P, G):
        issue(range(b, b + G))
    issued = P
    for i in range(nbytes):
        if i % G == 0:
            for b in issue(range(i + P, i + P + G)):
                issued = b + 1
            lines.append(f"s_waitcnt lgkmcnt({issued - (i + G)})")
        hin = H1 if i % 2 == 0 else H0
        hout = H0 if i % 2 == 0 else H1
        lines.append(f"v_alignbit_b32 {hout}, {hin}, {hin}, 31")
        lines.append(f"v_bitop3_b32 {hout}, {hout}, %{leave(i)}, %{enter(i)} bitop3:0x96")
        if i % 2 == 1:
            if i == 1 and acc_init:
                lines.append(f"v_max_u32 {ACC}, {H0}, {H1}")
            else:
                lines.append(f"v_max3_u32 {ACC}, {ACC}, {H0}, {H1}")
    return "\\n\\t".join(lines), nd


def emit(name, nbytes, enter, leave, G, P):
    asm, nd = body(nbytes, enter, leave, G, P, True)
    outs = [f'"+v"(R[{i}])' for i in range(128)] + ['"+v"(h)', '"=&v"(acc)', '"=&v"(h0)'] + \
           [f'"=&v"(a{k})' for k in range(NA)]
    ins = [f'"v"(d[{w}])' for w in range(nd)] + ['"v"(lanebase)'] + [f'"s"(sel{k})' for k in range(4)]
    return "\n".join([
        f"__device__ __forceinline__ uint32_t {name}(const uint32_t (&d)[{nd}], uint32_t (&R)[128],",
        "                                          uint32_t& h, uint32_t lanebase) {",
        "    uint32_t acc, h0, " + ", ".join(f"a{k}" for k in range(NA)) + ";",
        "    const uint32_t sel0 = 0x0c0c0400u, sel1 = 0x0c0c0500u, sel2 = 0x0c0c0600u, sel3 = 0x0c0c0700u;",
        "    asm volatile(",
        f'        "{asm}"',
        "        : " + ", ".join(outs),
        "        : " + ", ".join(ins),
        '        : "memory");',
        "    return acc;",
        "}", ""])


def body_f2(nbytes, enter, leave, G, P):
    """Parity-frame body (FRAME 2).  Byte i (u = i & 1) keeps g_i = rotl(h_i, c - u):
        u = 1:  g = g ^ T1[leave] ^ T1[enter]                (one v_bitop3)
        u = 0:  g = rotl(g, 2) ^ T0[leave] ^ T0[enter]       (v_alignbit + v_bitop3)
    with T0 = rotl(T, c) and T1 = rotl(T, c - 1) interleaved in each 256-byte table row
    (32 replicas each; ds_read_b32 banks by (a/4) % 32 per 32-lane half, so 32 replicas
    are conflict-free).  Byte i-64 has the same parity, so its ring slot already holds
    the right variant.  3 VALU per byte instead of 3.5.  Operands as body() but with two
    lane bases: LB0 (even bytes), LB1 (odd bytes)."""
    nd = nbytes // 4
    H1, ACC, H0 = "%128", "%129", "%130"
    A = lambda k: f"%{131 + k}"
    D = lambda w: f"%{131 + NA + w}"
    LB = lambda u: f"%{131 + NA + nd + u}"
    S = lambda k: f"%{131 + NA + nd + 2 + k}"
    assert P + G <= 15 and G in (2, 4) and P % G == 0
    lines = ["s_waitcnt lgkmcnt(0)"]

    def issue(bs):
        bs = [b for b in bs if b < nbytes]
        for b in bs:
            lines.append(f"v_perm_b32 {A(b % NA)}, {D(b // 4)}, {LB(b % 2)}, {S(b % 4)}")
        for b in bs:
            lines.append(f"ds_read_b32 %{enter(b)}, {A(b % NA)}")
        return bs

    for b in range(0, P, G):
        issue(range(b, b + G))
    issued = P
    for i in range(nbytes):
        if i % G == 0:
            for b in issue(range(i + P, i + P + G)):
                issued = b + 1
            lines.append(f"s_waitcnt lgkmcnt({issued - (i + G)})")
        if i % 2 == 0:  # H1 holds g_{i-1}; g_i -> H0
            lines.append(f"v_alignbit_b32 {H0}, {H1}, {H1}, 30")
            lines.append(f"v_bitop3_b32 {H0}, {H0}, %{leave(i)}, %{enter(i)} bitop3:0x96")
        else:
            lines.append(f"v_bitop3_b32 {H1}, {H0}, %{leave(i)}, %{enter(i)} bitop3:0x96")
            if i == 1:
                lines.append(f"v_max_u32 {ACC}, {H0}, {H1}")
            else:
                lines.append(f"v_max3_u32 {ACC}, {ACC}, {H0}, {H1}")
    return "\\n\\t".join(lines), nd


def emit_f2(name, nbytes, enter, leave, G, P):
    asm, nd = body_f2(nbytes, enter, leave, G, P)
    outs = [f'"+v"(R[{i}])' for i in range(128)] + ['"+v"(h)', '"=&v"(acc)', '"=&v"(h0)'] + \
           [f'"=&v"(a{k})' for k in range(NA)]
    ins = [f'"v"(d[{w}])' for w in range(nd)] + ['"v"(lb0)', '"v"(lb1)'] + [f'"s"(sel{k})' for k in range(4)]
    return "\n".join([
        f"__device__ __forceinline__ uint32_t {name}(const uint32_t (&d)[{nd}], uint32_t (&R)[128],",
        "                                          uint32_t& h, uint32_t lb0, uint32_t lb1) {",
        "    uint32_t acc, h0, " + ", ".join(f"a{k}" for k in range(NA)) + ";",
        "    const uint32_t sel0 = 0x0c0c0400u, sel1 = 0x0c0c0500u, sel2 = 0x0c0c0600u, sel3 = 0x0c0c0700u;",
        "    asm volatile(",
        f'        "{asm}"',
        "        : " + ", ".join(outs),
        "        : " + ", ".join(ins),
        '        : "memory");',
        "    return acc;",
        "}", ""])


def body_ring(nring, nbytes, enter, leave, G, P):
    """Parity-frame body over a ring of `nring` registers (the R96 kernel: 96 slots,
    byte i of phase p enters slot (128p + i) % 96 and leaves slot (128p + i + 32) % 96,
    so three 128-byte phases repeat).  Same per-byte ops as body_f2."""
    nd = nbytes // 4
    H1, ACC, H0 = f"%{nring}", f"%{nring + 1}", f"%{nring + 2}"
    b0 = nring + 3
    A = lambda k: f"%{b0 + k}"
    D = lambda w: f"%{b0 + NA + w}"
    LB = lambda u: f"%{b0 + NA + nd + u}"
    S = lambda k: f"%{b0 + NA + nd + 2 + k}"
    assert P + G <= 15 and G in (2, 4) and P % G == 0 and P <= nring - 64
    lines = ["s_waitcnt lgkmcnt(0)"]

    def issue(bs):
        bs = [b for b in bs if b < nbytes]
        for b in bs:
            lines.append(f"v_perm_b32 {A(b % NA)}, {D(b // 4)}, {LB(b % 2)}, {S(b % 4)}")
        for b in bs:
            lines.append(f"ds_read_b32 %{enter(b)}, {A(b % NA)}")
        return bs

    for b in range(0, P, G):
        issue(range(b, b + G))
    issued = P
    for i in range(nbytes):
        if i % G == 0:
            for b in issue(range(i + P, i + P + G)):
                issued = b + 1
            lines.append(f"s_waitcnt lgkmcnt({issued - (i + G)})")
        if i % 2 == 0:
            lines.append(f"v_alignbit_b32 {H0}, {H1}, {H1}, 30")
            lines.append(f"v_bitop3_b32 {H0}, {H0}, %{leave(i)}, %{enter(i)} bitop3:0x96")
        else:
            lines.append(f"v_bitop3_b32 {H1}, {H0}, %{leave(i)}, %{enter(i)} bitop3:0x96")
            if i == 1:
                lines.append(f"v_max_u32 {ACC}, {H0}, {H1}")
            else:
                lines.append(f"v_max3_u32 {ACC}, {ACC}, {H0}, {H1}")
    return "\\n\\t".join(lines), nd


def emit_ring(name, nring, phase, G, P):
    ent = lambda i: (128 * phase + i) % nring
    lv = lambda i: (128 * phase + i + nring - 64) % nring
    asm, nd = body_ring(nring, 128, ent, lv, G, P)
    outs = [f'"+v"(R[{i}])' for i in range(nring)] + ['"+v"(h)', '"=&v"(acc)', '"=&v"(h0)'] + \
           [f'"=&v"(a{k})' for k in range(NA)]
    ins = [f'"v"(d[{w}])' for w in range(nd)] + ['"v"(lb0)', '"v"(lb1)'] + [f'"s"(sel{k})' for k in range(4)]
    return "\n".join([
        f"__device__ __forceinline__ uint32_t {name}(const uint32_t (&d)[{nd}], uint32_t (&R)[{nring}],",
        "                                          uint32_t& h, uint32_t lb0, uint32_t lb1) {",
        "    uint32_t acc, h0, " + ", ".join(f"a{k}" for k in range(NA)) + ";",
        "    const uint32_t sel0 = 0x0c0c0400u, sel1 = 0x0c0c0500u, sel2 = 0x0c0c0600u, sel3 = 0x0c0c0700u;",
        "    asm volatile(",
        f'        "{asm}"',
        "        : " + ", ".join(outs),
        "        : " + ", ".join(ins),
        '        : "memory");',
        "    return acc;",
        "}", ""])


def main():
    out = ["// GENERATED by gen_roll_asm.py -- do not edit by hand.",
           "// Hand-scheduled bodies of the rolling-hash loop (see the generator's docstring).",
           "#pragma once", ""]
    # 128-byte iteration: byte i enters slot i, leaves slot (i+64)%128
    ent = lambda i: i
    lv = lambda i: (i + 64) % 128
    out.append("// 128-byte iteration, waits per 2 bytes, 12 reads ahead")
    out.append(emit("roll128_asm", 128, ent, lv, 2, 12))
    out.append("// 128-byte iteration, waits per 4 bytes, 8 reads ahead")
    out.append(emit("roll128_asm_g4", 128, ent, lv, 4, 8))
    out.append("// 128-byte iteration, parity frame (3 VALU/byte), waits per 4 bytes, 8 reads ahead")
    out.append(emit_f2("roll128_asm_f2", 128, ent, lv, 4, 8))
    out.append("// parity frame, waits per 2 bytes, 12 / 10 reads ahead")
    out.append(emit_f2("roll128_asm_f2_g2p12", 128, ent, lv, 2, 12))
    out.append(emit_f2("roll128_asm_f2_g2p10", 128, ent, lv, 2, 10))
    out.append("// parity frame over a 96-register ring: three 128-byte phases (R96 kernel)")
    for ph in range(3):
        out.append(emit_ring(f"roll128_r96_p{ph}", 96, ph, 4, 8))
    # 64-byte halves of the 128-entry ring (v2 kernel)
    out.append("// 64-byte halves of the 128-entry ring")
    out.append(emit("roll64_asm_h0", 64, lambda i: i, lambda i: 64 + i, 2, 12))
    out.append(emit("roll64_asm_h1", 64, lambda i: 64 + i, lambda i: i, 2, 12))
    sys.stdout.write("\n".join(out))


if __name__ == "__main__":
    main()
