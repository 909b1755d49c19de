"""Experiment transform (tools/exp_build.sh): per-wave s_memtime stamps in gcn_fwd_pow_kernel,
written past the BN partial slots of the probe's buffer (tools/gcn_probe.py --stamps):
per wave [hw_id, t_entry, t_staged, t_support0, t_support1, t_support2, t_end, xcc_id] (low 32 bits)."""
import sys
p = sys.argv[1]
s = open(p).read()
a = '''  GPair q0 = (u.k1 > u.k0) ? gp_load(src, 0) : GPair{};
  // piece 0's'''
b = '''  unsigned stt[8];
  stt[1] = (unsigned)__builtin_amdgcn_s_memtime();
  GPair q0 = (u.k1 > u.k0) ? gp_load(src, 0) : GPair{};
  // piece 0's'''
assert a in s; s = s.replace(a, b)
a = '''  global_to_lds(hs, ldh, n, pow_img_rows(np), xs);
  __syncthreads();
  f32x16 hacc = zero16();'''
b = '''  global_to_lds(hs, ldh, n, pow_img_rows(np), xs);
  __syncthreads();
  stt[2] = (unsigned)__builtin_amdgcn_s_memtime();
  f32x16 hacc = zero16();'''
assert a in s; s = s.replace(a, b)
a = '''        acc_to_global(hs + (2 + 2 * k) * CH, ldh, d2, w0, lane, n);
      }
    }
  };'''
b = '''        acc_to_global(hs + (2 + 2 * k) * CH, ldh, d2, w0, lane, n);
      }
    }
    stt[3 + (k < 3 ? k : 2)] = (unsigned)__builtin_amdgcn_s_memtime();
  };'''
assert a in s; s = s.replace(a, b)
a = '''  if (tile_epi) {
    fwd_tile_epilogue(a, hacc, res, row0, w0, lane, n, u.slice, wave, nkb);
    return;
  }'''
b = '''  if (tile_epi) {
    fwd_tile_epilogue(a, hacc, res, row0, w0, lane, n, u.slice, wave, nkb);
    stt[6] = (unsigned)__builtin_amdgcn_s_memtime();
    if (lane == 0) {
      unsigned* dg = (unsigned*)(a.bn_part + (long)a.slices * nkb * 3 * CH) + 8 * (blockIdx.x * (blockDim.x >> 6) + wave);
      dg[0] = __builtin_amdgcn_s_getreg(63492);
      for (int q = 1; q < 7; ++q) dg[q] = stt[q];
      dg[7] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
    return;
  }'''
assert a in s; s = s.replace(a, b)
open(p, 'w').write(s)
