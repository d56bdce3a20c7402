// audio.hip -- the data path either side of the mel engine, gfx950.
//
// Log-mel extraction and Griffin-Lim inversion, Tacotron2 convention (n_fft 1024, hop 256,
// periodic Hann, centre reflect padding, 80 Slaney mel bands).  The transforms themselves
// are tt2_gemm calls in f32 (the window-folded DFT / inverse-DFT bases and the mel
// filterbank are small dense matrices); these kernels are the byte-moving steps around
// them.  Frame layout: utterance b's padded signal occupies padded[b * Lp, (b + 1) * Lp)
// with Lp a multiple of the hop, so the frames of the WHOLE batch are one strided matrix
// (row r starts at sample r * hop, ld = hop, rows overlap) and utterance b owns rows
// [b * R, b * R + n_frames_b), R = Lp / hop.  The few rows that straddle two utterances
// are computed and never read.
#include <math.h>

#include "tt2_capi.h"
#include "tt2_internal.h"
#include "tt2_common.h"

namespace {
constexpr int NT = 256;

int grid_for(int64_t total) {
  const int64_t b = (total + NT - 1) / NT;
  return (int)(b < 16384 ? (b > 0 ? b : 1) : 16384);
}

// padded[b][j] = x[b][reflect(j - pad)] for j < len_b + 2 pad, 0 beyond (np.pad mode "reflect")
__global__ void reflect_pad_kernel(const float* x, int64_t ldx, const int32_t* lens, int B, int L, float* out,
                                   int64_t Lp, int pad) {
  const int64_t total = (int64_t)B * Lp;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int b = (int)(i / Lp);
    const int j = (int)(i - (int64_t)b * Lp);
    const int len = lens ? min(lens[b], L) : L;
    int s = j - pad;
    float v = 0.f;
    if (s < len + pad && len > 0) {
      if (s < 0) s = -s;
      if (s >= len) s = 2 * (len - 1) - s;
      s = min(max(s, 0), len - 1);   // lengths <= pad: clamp (never read out of bounds)
      v = x[(int64_t)b * ldx + s];
    }
    out[i] = v;
  }
}

// mag[r][k] = |spec[r][k] + i spec[r][nb + k]| for k < nb; 0 for nb <= k < ldm
__global__ void spec_mag_kernel(const float* spec, int64_t lds, int M, int nb, float* mag, int64_t ldm) {
  const int64_t total = (int64_t)M * ldm;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t r = i / ldm;
    const int k = (int)(i - r * ldm);
    float v = 0.f;
    if (k < nb) {
      const float re = spec[r * lds + k], im = spec[r * lds + nb + k];
      v = sqrtf(re * re + im * im);
    }
    mag[i] = v;
  }
}

// out[r][k], out[r][nb + k] = mag[r][k] * e / |e| (e = est[r][k] + i est[r][nb + k]; phase 0
// where est is null or e == 0); padding columns [2 nb, ldo) zeroed
__global__ void spec_rephase_kernel(const float* mag, int64_t ldm, const float* est, int64_t lde, int M, int nb,
                                    float* out, int64_t ldo) {
  const int64_t total = (int64_t)M * nb;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t r = i / nb;
    const int k = (int)(i - r * nb);
    const float m = mag[r * ldm + k];
    float c = 1.f, s = 0.f;
    if (est) {
      const float re = est[r * lde + k], im = est[r * lde + nb + k];
      const float a = sqrtf(re * re + im * im);
      if (a > 0.f) { c = re / a; s = im / a; }
    }
    out[r * ldo + k] = m * c;
    out[r * ldo + nb + k] = m * s;
    if (k < ldo - 2 * nb) out[r * ldo + 2 * nb + k] = 0.f;
  }
}

// Least-squares overlap-add (the iSTFT's second half): frames[b * R + f][n] (already
// multiplied by the synthesis window) summed into y[b][i] for i < len_b, divided by the
// summed squared window of the frames that cover sample i + pad; 0 for i >= len_b.
__global__ void overlap_add_kernel(const float* frames, int64_t ldf, const int32_t* lens, int B, int L, int R,
                                   int n_fft, int hop, int pad, float* y, int64_t ldy) {
  const int64_t total = (int64_t)B * L;
  const float w0 = 6.283185307179586f / (float)n_fft;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int b = (int)(i / L);
    const int t = (int)(i - (int64_t)b * L);
    const int len = lens ? min(lens[b], L) : L;
    float v = 0.f;
    if (t < len) {
      const int nf = 1 + len / hop;
      const int j = t + pad;                       // position in the padded signal
      int f0 = (j - n_fft + hop) / hop;            // first frame with f * hop + n_fft > j
      if (f0 < 0) f0 = 0;
      const int f1 = min(nf - 1, j / hop);
      float acc = 0.f, wss = 0.f;
      for (int f = f0; f <= f1; ++f) {
        const int n = j - f * hop;
        const float w = 0.5f - 0.5f * cosf(w0 * (float)n);
        acc += frames[((int64_t)b * R + f) * ldf + n];
        wss += w * w;
      }
      v = wss > 1e-8f ? acc / wss : 0.f;
    }
    y[(int64_t)b * ldy + t] = v;
  }
}

// dir 0 (gather): out[b][t][c] = log(max(rows[b * R + t][c], clamp)) for t < nf_b, log(clamp)
//                 beyond (silence);  dir 1 (scatter): rows[b * R + t][c] = exp(mel[b][t][c]) for
//                 t < nf_b, 0 beyond.  nf_b = frames[b] (or T).
__global__ void mel_rows_kernel(float* rows, int64_t ldr, float* mel, const int32_t* frames, int B, int T, int C,
                                int R, float clamp, int dir) {
  const int64_t total = (int64_t)B * R * C;
  const float lc = logf(clamp);
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int c = (int)(i % C);
    const int64_t rr = i / C;
    const int b = (int)(rr / R), t = (int)(rr - (int64_t)b * R);
    const int nf = frames ? min(frames[b], T) : T;
    if (dir == 0) {
      if (t < T) mel[((int64_t)b * T + t) * C + c] = t < nf ? logf(fmaxf(rows[rr * ldr + c], clamp)) : lc;
    } else {
      rows[rr * ldr + c] = t < nf ? expf(mel[((int64_t)b * T + t) * C + c]) : 0.f;
    }
  }
}

}  // namespace

extern "C" int tt2_reflect_pad(const float* x, int64_t ldx, const int32_t* lens, int32_t batch, int32_t len,
                               float* out, int64_t padded_len, int32_t pad, hipStream_t s) {
  if (!x || !out || batch <= 0 || len <= 0) return tt2_set_error(TT2_E_INVALID, "tt2_reflect_pad: bad args");
  if (pad >= len) return tt2_set_error(TT2_E_INVALID, "tt2_reflect_pad: pad must be < length");
  if (padded_len < (int64_t)len + 2 * pad) return tt2_set_error(TT2_E_INVALID, "tt2_reflect_pad: padded_len short");
  hipLaunchKernelGGL(reflect_pad_kernel, dim3(grid_for((int64_t)batch * padded_len)), dim3(NT), 0, s, x, ldx, lens,
                     batch, len, out, padded_len, pad);
  return tt2_check_launch(hipGetLastError(), "tt2_reflect_pad");
}

extern "C" int tt2_spec_magnitude(const float* spec, int64_t ld_spec, int32_t m, int32_t n_bins, float* mag,
                                  int64_t ld_mag, hipStream_t s) {
  if (!spec || !mag || m <= 0 || ld_spec < 2 * n_bins || ld_mag < n_bins)
    return tt2_set_error(TT2_E_INVALID, "tt2_spec_magnitude: bad args");
  hipLaunchKernelGGL(spec_mag_kernel, dim3(grid_for((int64_t)m * ld_mag)), dim3(NT), 0, s, spec, ld_spec, m, n_bins,
                     mag, ld_mag);
  return tt2_check_launch(hipGetLastError(), "tt2_spec_magnitude");
}

extern "C" int tt2_spec_rephase(const float* mag, int64_t ld_mag, const float* est, int64_t ld_est, int32_t m,
                                int32_t n_bins, float* out, int64_t ld_out, hipStream_t s) {
  if (!mag || !out || m <= 0 || ld_out < 2 * n_bins || ld_out > 3 * n_bins || (est && ld_est < 2 * n_bins))
    return tt2_set_error(TT2_E_INVALID, "tt2_spec_rephase: bad args");
  hipLaunchKernelGGL(spec_rephase_kernel, dim3(grid_for((int64_t)m * n_bins)), dim3(NT), 0, s, mag, ld_mag, est,
                     ld_est, m, n_bins, out, ld_out);
  return tt2_check_launch(hipGetLastError(), "tt2_spec_rephase");
}

extern "C" int tt2_overlap_add(const float* frames, int64_t ld_frames, const int32_t* lens, int32_t batch,
                               int32_t len, int32_t rows_per_utt, int32_t n_fft, int32_t hop, float* y, int64_t ld_y,
                               hipStream_t s) {
  if (!frames || !y || batch <= 0 || len <= 0 || hop <= 0 || n_fft < hop || ld_frames < n_fft ||
      (int64_t)rows_per_utt * hop < (int64_t)len + n_fft)
    return tt2_set_error(TT2_E_INVALID, "tt2_overlap_add: bad args");
  hipLaunchKernelGGL(overlap_add_kernel, dim3(grid_for((int64_t)batch * len)), dim3(NT), 0, s, frames, ld_frames,
                     lens, batch, len, rows_per_utt, n_fft, hop, n_fft / 2, y, ld_y);
  return tt2_check_launch(hipGetLastError(), "tt2_overlap_add");
}

extern "C" int tt2_mel_rows(float* rows, int64_t ld_rows, float* mel, const int32_t* frames, int32_t batch,
                            int32_t t, int32_t n_mels, int32_t rows_per_utt, float clamp, int32_t scatter,
                            hipStream_t s) {
  if (!rows || !mel || batch <= 0 || t <= 0 || t > rows_per_utt || ld_rows < n_mels || clamp <= 0.f)
    return tt2_set_error(TT2_E_INVALID, "tt2_mel_rows: bad args");
  hipLaunchKernelGGL(mel_rows_kernel, dim3(grid_for((int64_t)batch * rows_per_utt * n_mels)), dim3(NT), 0, s, rows,
                     ld_rows, mel, frames, batch, t, n_mels, rows_per_utt, clamp, scatter ? 1 : 0);
  return tt2_check_launch(hipGetLastError(), "tt2_mel_rows");
}
