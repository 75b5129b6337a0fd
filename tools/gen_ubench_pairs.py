#!/usr/bin/env python3
"""Generate tools/ubench_pairs.hip: issue-rate probes for instruction
pairs/sequences on gfx950 (which VALU ops dual-issue, and when).

Each case is a list of asm lines executed per iteration (16x unrolled);
registers a0..a7 are independent chains, b/c are read-only inputs, s is an
SGPR.  Reported: wave-instructions per CU-cycle (1.0 = one per cycle per
CU, i.e. one wave64 instruction per 4 cycles per SIMD)."""
import os

CASES = [
    ("xor x8 indep", ["v_xor_b32 {a%d}, {a%d}, {b}" % (i, i) for i in range(8)]),
    ("xor x1 chain", ["v_xor_b32 {a0}, {a0}, {b}"] * 8),
    ("xor x2 chains", ["v_xor_b32 {a%d}, {a%d}, {b}" % (i % 2, i % 2) for i in range(8)]),
    ("xor x4 chains", ["v_xor_b32 {a%d}, {a%d}, {b}" % (i % 4, i % 4) for i in range(8)]),
    ("add_lit x8", ["v_add_u32 {a%d}, 0x12345678, {a%d}" % (i, i) for i in range(8)]),
    ("add_inl x8", ["v_add_u32 {a%d}, 5, {a%d}" % (i, i) for i in range(8)]),
    ("add_sgpr x8", ["v_add_u32 {a%d}, {s}, {a%d}" % (i, i) for i in range(8)]),
    ("lshl_e32v x8", ["v_lshlrev_b32 {a%d}, {b}, {a%d}" % (i, i) for i in range(8)]),
    ("lshl_e32c x8", ["v_lshlrev_b32 {a%d}, 3, {a%d}" % (i, i) for i in range(8)]),
    ("lshl_e64v x8", ["v_lshlrev_b32_e64 {a%d}, {b}, {a%d}" % (i, i) for i in range(8)]),
    ("lshr_e32c x8", ["v_lshrrev_b32 {a%d}, 3, {a%d}" % (i, i) for i in range(8)]),
    ("lshr_e32v x8", ["v_lshrrev_b32 {a%d}, {b}, {a%d}" % (i, i) for i in range(8)]),
    ("ashr x8", ["v_ashrrev_i32 {a%d}, 3, {a%d}" % (i, i) for i in range(8)]),
    ("xor+add x4", sum([["v_xor_b32 {a%d}, {a%d}, {b}" % (2 * i, 2 * i),
                         "v_add_u32 {a%d}, {a%d}, {b}" % (2 * i + 1, 2 * i + 1)] for i in range(4)], [])),
    ("bitop3+add x4", sum([["v_bitop3_b32 {a%d}, {a%d}, {b}, {c} bitop3:0x96" % (2 * i, 2 * i),
                            "v_add_u32 {a%d}, {a%d}, {b}" % (2 * i + 1, 2 * i + 1)] for i in range(4)], [])),
    ("bitop3 3src x8", ["v_bitop3_b32 {a%d}, {a%d}, {b}, {c} bitop3:0xca" % (i, i) for i in range(8)]),
    ("bitop3 dep-pairs", sum([["v_bitop3_b32 {a%d}, {a%d}, {b}, {c} bitop3:0x96" % (i, i),
                               "v_bitop3_b32 {a%d}, {a%d}, {b}, {c} bitop3:0xca" % (i, i)] for i in range(4)], [])),
    ("alignbit+alignbit", ["v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i, i, i) for i in range(8)]),
    ("alignbit,xor,xor", sum([["v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i, i, i),
                               "v_xor_b32 {a%d}, {a%d}, {b}" % ((i + 4) % 8, (i + 4) % 8),
                               "v_xor_b32 {a%d}, {a%d}, {c}" % ((i + 5) % 8, (i + 5) % 8)] for i in range(0, 8, 2)], [])),
    ("add3 x8", ["v_add3_u32 {a%d}, {a%d}, {b}, {c}" % (i, i) for i in range(8)]),
    ("sub x8", ["v_sub_u32 {a%d}, {a%d}, {b}" % (i, i) for i in range(8)]),
    ("mov x8", ["v_mov_b32 {a%d}, {b}" % i for i in range(8)]),
    ("add_same_src x8", ["v_add_u32 {a%d}, {b}, {c}" % i for i in range(8)]),
    # SGPR operands on ops that are slow anyway (the search loop's K constants sit in SGPRs)
    ("add3_sgpr x8", ["v_add3_u32 {a%d}, {a%d}, {b}, {s}" % (i, i) for i in range(8)]),
    ("bitop3_sgpr x8", ["v_bitop3_b32 {a%d}, {a%d}, {b}, {s} bitop3:0x96" % (i, i) for i in range(8)]),
    ("alignbit_sgpr x8", ["v_alignbit_b32 {a%d}, {s}, {s}, 7" % i for i in range(8)]),
    ("add3,xor,xor", sum([["v_add3_u32 {a%d}, {a%d}, {b}, {c}" % (i, i),
                           "v_xor_b32 {a%d}, {a%d}, {b}" % ((i + 4) % 8, (i + 4) % 8),
                           "v_xor_b32 {a%d}, {a%d}, {c}" % ((i + 5) % 8, (i + 5) % 8)] for i in range(0, 8, 2)], [])),
    ("add3_sgpr,xor,xor", sum([["v_add3_u32 {a%d}, {a%d}, {b}, {s}" % (i, i),
                                "v_xor_b32 {a%d}, {a%d}, {b}" % ((i + 4) % 8, (i + 4) % 8),
                                "v_xor_b32 {a%d}, {a%d}, {c}" % ((i + 5) % 8, (i + 5) % 8)] for i in range(0, 8, 2)], [])),
    ("add3,alignbit", sum([["v_add3_u32 {a%d}, {a%d}, {b}, {c}" % (i, i),
                            "v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i + 1, i + 1, i + 1)] for i in range(0, 8, 2)], [])),
    ("add3_sgpr,alignbit", sum([["v_add3_u32 {a%d}, {a%d}, {b}, {s}" % (i, i),
                                 "v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i + 1, i + 1, i + 1)] for i in range(0, 8, 2)], [])),
    # wave priority around slow / fast runs (s_setprio): does it let fast ops co-issue?
    ("prio S0 F2: a,x,x", sum([["s_setprio 0", "v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i, i, i), "s_setprio 2",
                                "v_xor_b32 {a%d}, {a%d}, {b}" % ((i + 4) % 8, (i + 4) % 8),
                                "v_xor_b32 {a%d}, {a%d}, {c}" % ((i + 5) % 8, (i + 5) % 8)] for i in range(0, 8, 2)], [])),
    ("prio S2 F0: a,x,x", sum([["s_setprio 2", "v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i, i, i), "s_setprio 0",
                                "v_xor_b32 {a%d}, {a%d}, {b}" % ((i + 4) % 8, (i + 4) % 8),
                                "v_xor_b32 {a%d}, {a%d}, {c}" % ((i + 5) % 8, (i + 5) % 8)] for i in range(0, 8, 2)], [])),
    ("runs 4S 8F", ["v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i, i, i) for i in range(4)] +
                   ["v_xor_b32 {a%d}, {a%d}, {b}" % (4 + i % 4, 4 + i % 4) for i in range(8)]),
    ("prio runs 4S 8F", ["s_setprio 0"] + ["v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i, i, i) for i in range(4)] +
                        ["s_setprio 2"] + ["v_xor_b32 {a%d}, {a%d}, {b}" % (4 + i % 4, 4 + i % 4) for i in range(8)]),
    # one SHA-256 round + schedule word as grouped runs: 10 S (rotates), 9 F (xor3/shr/add/Ch/Maj),
    # 4 S (add3), 1 F (e = d + T1); with and without priority toggles
    ("sha grp S10F9S4F1", ["v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i % 8, i % 8, i % 8) for i in range(10)] +
                          ["v_bitop3_b32 {a%d}, {a%d}, {b}, {c} bitop3:0x96" % (i % 8, i % 8) for i in range(9)] +
                          ["v_add3_u32 {a%d}, {a%d}, {b}, {c}" % (i % 8, i % 8) for i in range(4)] +
                          ["v_add_u32 {a0}, {a0}, {b}"]),
    ("sha grp prio", ["s_setprio 2"] + ["v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i % 8, i % 8, i % 8) for i in range(10)] +
                     ["s_setprio 0"] + ["v_bitop3_b32 {a%d}, {a%d}, {b}, {c} bitop3:0x96" % (i % 8, i % 8) for i in range(9)] +
                     ["s_setprio 2"] + ["v_add3_u32 {a%d}, {a%d}, {b}, {c}" % (i % 8, i % 8) for i in range(4)] +
                     ["s_setprio 0", "v_add_u32 {a0}, {a0}, {b}"]),
    ("sha grp prio3", ["s_setprio 3"] + ["v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i % 8, i % 8, i % 8) for i in range(10)] +
                      ["s_setprio 0"] + ["v_bitop3_b32 {a%d}, {a%d}, {b}, {c} bitop3:0x96" % (i % 8, i % 8) for i in range(9)] +
                      ["s_setprio 3"] + ["v_add3_u32 {a%d}, {a%d}, {b}, {c}" % (i % 8, i % 8) for i in range(4)] +
                      ["s_setprio 0", "v_add_u32 {a0}, {a0}, {b}"]),
    ("prio runs 4S2 8F0", ["s_setprio 2"] + ["v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i, i, i) for i in range(4)] +
                          ["s_setprio 0"] + ["v_xor_b32 {a%d}, {a%d}, {b}" % (4 + i % 4, 4 + i % 4) for i in range(8)]),
    # the loop's actual interleaving (S,S,S,F,F,S,S,S,S,F,...) as compiled
    ("sha fine", ["v_alignbit_b32 {a0}, {a0}, {a0}, 25", "v_alignbit_b32 {a1}, {a1}, {a1}, 11",
                  "v_alignbit_b32 {a2}, {a2}, {a2}, 6", "v_bitop3_b32 {a3}, {a3}, {b}, {c} bitop3:0x96",
                  "v_bitop3_b32 {a4}, {a4}, {b}, {c} bitop3:0xca", "v_add3_u32 {a5}, {a5}, {b}, {c}",
                  "v_add3_u32 {a6}, {a6}, {b}, {c}", "v_alignbit_b32 {a7}, {a7}, {a7}, 22",
                  "v_alignbit_b32 {a0}, {a0}, {a0}, 13", "v_alignbit_b32 {a1}, {a1}, {a1}, 2",
                  "v_bitop3_b32 {a2}, {a2}, {b}, {c} bitop3:0x96", "v_bitop3_b32 {a3}, {a3}, {b}, {c} bitop3:0xe8",
                  "v_add_u32 {a4}, {a4}, {b}", "v_add3_u32 {a5}, {a5}, {b}, {c}",
                  "v_lshrrev_b32 {a6}, 3, {a6}", "v_alignbit_b32 {a7}, {a7}, {a7}, 18",
                  "v_alignbit_b32 {a0}, {a0}, {a0}, 7", "v_bitop3_b32 {a1}, {a1}, {b}, {c} bitop3:0x96",
                  "v_alignbit_b32 {a2}, {a2}, {a2}, 17", "v_alignbit_b32 {a3}, {a3}, {a3}, 19",
                  "v_lshrrev_b32 {a4}, 10, {a4}", "v_bitop3_b32 {a5}, {a5}, {b}, {c} bitop3:0x96",
                  "v_add_u32 {a6}, {a6}, {b}", "v_add3_u32 {a7}, {a7}, {b}, {c}"]),
    ("nop-only SALU a,x,x",sum([["s_nop 0", "v_alignbit_b32 {a%d}, {a%d}, {a%d}, 7" % (i, i, i), "s_nop 0",
                                  "v_xor_b32 {a%d}, {a%d}, {b}" % ((i + 4) % 8, (i + 4) % 8),
                                  "v_xor_b32 {a%d}, {a%d}, {c}" % ((i + 5) % 8, (i + 5) % 8)] for i in range(0, 8, 2)], [])),
]


def reg(name):
    return "%[" + name + "]"


def emit():
    out = ['// generated by tools/gen_ubench_pairs.py -- do not edit',
           '#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdlib>',
           '#define ITERS 4096', '']
    names = []
    for ci, (name, lines) in enumerate(CASES):
        names.append(name)
        body = "\\n\\t".join(l.format(**{f"a{i}": reg(f"a{i}") for i in range(8)}, b=reg("b"), c=reg("c"),
                                         s=reg("s")) for l in lines)
        out.append(f'__global__ __launch_bounds__(256) void k{ci}(unsigned* out, unsigned long long* clk, unsigned seed) {{')
        out.append('  unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;')
        out.append('  unsigned b = seed * 3 + threadIdx.x, c = b ^ 0x5555;')
        out.append('  unsigned s = __builtin_amdgcn_readfirstlane(seed * 7);')
        out.append('  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();')
        out.append('  for (int i = 0; i < ITERS; ++i) {')
        for _ in range(16):
            out.append(f'    asm volatile("{body}" : [a0]"+v"(a0), [a1]"+v"(a1), [a2]"+v"(a2), [a3]"+v"(a3), '
                       f'[a4]"+v"(a4), [a5]"+v"(a5), [a6]"+v"(a6), [a7]"+v"(a7) : [b]"v"(b), [c]"v"(c), [s]"s"(s) : "vcc");')
        out.append('  }')
        out.append('  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();')
        out.append('  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;')
        out.append('  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }')
        out.append('}')
    out.append('typedef void (*kfn)(unsigned*, unsigned long long*, unsigned);')
    out.append('static kfn ks[] = {' + ", ".join(f"k{i}" for i in range(len(CASES))) + '};')
    out.append('static const char* names[] = {' + ", ".join('"%s"' % n for n in names) + '};')
    out.append('static const int ninstr[] = {' + ", ".join(str(sum(1 for x in l if x.startswith("v_"))) for _, l in CASES) + '};')
    out.append('''
int main(int argc, char** argv) {
  int bpc = argc > 1 ? atoi(argv[1]) : 8;
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  int grid = p.multiProcessorCount * bpc;
  unsigned* out; unsigned long long* clk;
  (void)hipMalloc(&out, (size_t)grid * 256 * 4);
  (void)hipMalloc(&clk, (size_t)grid * 16);
  unsigned long long* h = (unsigned long long*)malloc((size_t)grid * 16);
  printf("%s %d CUs, %d blocks/CU\\n", p.gcnArchName, p.multiProcessorCount, bpc);
  for (int c = 0; c < (int)(sizeof(ks) / sizeof(ks[0])); ++c) {
    ks[c]<<<grid, 256>>>(out, clk, 1);
    (void)hipDeviceSynchronize();
    ks[c]<<<grid, 256>>>(out, clk, 2);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, clk, (size_t)grid * 16, hipMemcpyDeviceToHost);
    double cyc = 0;
    for (int i = 0; i < grid; ++i) cyc += h[2 * i];
    cyc /= grid;  // shader cycles per workgroup lifetime
    double instr = (double)ITERS * 16 * ninstr[c] * 4 * bpc;  // wave-instrs per CU (4 waves/WG)
    printf("%-20s %.3f wave-instr/clk/CU\\n", names[c], instr / cyc);
  }
  return 0;
}''')
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ubench_pairs.hip")
    open(path, "w").write(emit())
    print(path)
