"""Generates the hand-ordered softmax instruction stream of one 32-query x 64-key wave-tile of the
d <= 64 fp16 forward (round 5): 32 v_exp_f32 on the scores, 16 v_cvt_pk_f16_f32 into the packed P,
16 v_dot2c_f32_f16 row sums into four accumulators and the packed-P max tree (v_pk_maximum3_f16),
software-pipelined so no instruction reads a result issued fewer than `lag` pairs earlier.

Operands of the emitted asm string (inline-asm operand numbers; outputs come first):
  %0..%15   packed P dwords (outputs, "=&v")
  %16..%19  row-sum accumulators (in/out, "+v")
  %20       packed max of P (output, "=&v")
  %21..     exp temporaries ("=&v"), nt = 2*(lag+1) of them
  %(21+nt)..%(52+nt)  the 32 scores s (inputs, "v")
Without row sums ("nosums": the caller sums after its rebase check) there are no %16..%19: the packed
max is %16, the temporaries %17.., the scores %(17+nt)..
Usage: python tools/gen/softmax_stream.py LAG DLAG [nosums]  -> prints a C string literal"""
import sys


def stream(lag: int = 1, dlag: int = 1, sums: bool = True):
    nt = 2 * (lag + 1)
    nl = 4 if sums else 0  # row-sum operands
    S = lambda i: f"%{17 + nl + nt + i}"
    P = lambda k: f"%{k}"
    L = lambda x: f"%{16 + x}"
    M = f"%{16 + nl}"
    T = lambda i: f"%{17 + nl + (i % nt)}"
    out = []
    mx_done = -1  # P dwords folded into M so far (index of last)
    for k in range(16 + lag + dlag + 2):
        if k < 16:
            out.append(f"v_exp_f32 {T(2 * k)}, {S(2 * k)}")
            out.append(f"v_exp_f32 {T(2 * k + 1)}, {S(2 * k + 1)}")
        c = k - lag  # pair converted this step
        if 0 <= c < 16:
            out.append(f"v_cvt_pk_f16_f32 {P(c)}, {T(2 * c)}, {T(2 * c + 1)}")
        r = c - dlag  # pair summed / maxed this step
        if 0 <= r < 16:
            if sums:
                out.append(f"v_dot2c_f32_f16 {L(r % 4)}, 0x3c003c00, {P(r)}")
            # max tree: fold pairs two at a time
            if r == 1:
                out.append(f"v_pk_max_f16 {M}, {P(0)}, {P(1)}")
                mx_done = 1
            elif r >= 3 and r % 2 == 1:
                out.append(f"v_pk_maximum3_f16 {M}, {M}, {P(r - 1)}, {P(r)}")
                mx_done = r
    assert mx_done == 15
    return out, nt


if __name__ == "__main__":
    lag = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    dlag = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    sums = (sys.argv[3] != "nosums") if len(sys.argv) > 3 else True
    ins, nt = stream(lag, dlag, sums)
    print(f"// lag {lag}, dlag {dlag}: {len(ins)} instructions, {nt} temporaries")
    print('"' + "\\n\\t".join(ins) + '"')

