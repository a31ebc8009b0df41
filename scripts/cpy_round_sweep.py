"""Offline check of the test-backend-ops CPY f32 -> Q8_0 / Q4_0 comparison.

The device's CPY f32 -> Q8_0 restates quantize_row_q8_0_ref (ggml-quants.c:199-222: id = 1/(amax/127),
roundf = half away from zero); ggml-cpu's CPY calls the type's from_float, which for Q8_0 is the x86
quantize_row_q8_0 (ggml-cpu/arch/x86/quants.c:290-360: id = 127/amax, _mm256_round_ps = half to even).
Q4_0's from_float is the _ref quantizer on both sides (ggml-cpu/quants.c:25-27).
This sweeps test-backend-ops' CPY shapes (test-backend-ops.cpp:5586-5589: {256,4,4,4}, {256,2,3,4})
with uniform [-1, 1] inputs over many seeds and reports the NMSE test-backend-ops would compute
(both outputs dequantized, test-backend-ops.cpp:180-193) against its CPY bound 1e-6 (:2396-2398).
CPU only (oracle/liboracle.so).
"""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import qref

n_seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
worst = {}
diff_codes = {}
for shape in ((256, 4, 4, 4), (256, 2, 3, 4)):
    n = int(np.prod(shape))
    for seed in range(n_seeds):
        rng = np.random.default_rng(seed)
        x = rng.uniform(-1.0, 1.0, n).astype(np.float32)
        for t, name in ((qref.Q8_0, "q8_0"),):
            dev = qref.quantize_act(t, x, qref.ACT_REF)
            cpu = qref.quantize_act(t, x, qref.ACT_X86)
            e = qref.nmse(qref.dequantize(t, dev, n), qref.dequantize(t, cpu, n))
            k = (name, shape)
            worst[k] = max(worst.get(k, 0.0), e)
            d = np.frombuffer(dev.tobytes(), np.uint8).reshape(-1, 34)[:, 2:] != np.frombuffer(cpu.tobytes(), np.uint8).reshape(-1, 34)[:, 2:]
            diff_codes[k] = diff_codes.get(k, 0) + int(d.sum())
for k in worst:
    print(f"{k[0]} ne={list(k[1])}: seeds {n_seeds}, codes differing {diff_codes[k]} "
          f"({diff_codes[k] / (n_seeds * np.prod(k[1])):.2e} per element), worst NMSE {worst[k]:.3e} (bound 1e-6)")
