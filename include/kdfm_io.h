/* kdfm_io.h — C-ABI of libkdfm_io.so: the host-side audio data path that feeds the ver5 step.
 *
 * The reference reads LibriSpeech / GigaSpeech through NeMo's manifest datasets
 * (AudioToBPEDataset, reached from ctc_bpe_models.py:96-165; source absent from the reference, see
 * SURVEY.md §8(f) row 2): a JSONL manifest written by build_manifest_from_hf
 * (asr_train_diffm.py:31-88) / build_manifest_from_hf_gigaspeech (asr_train_diffm_GS.py:35-178)
 * names FLAC/WAV files that DataLoader workers (ctc_models.py:370-380, num_workers 8,
 * conformer_ctc_bpe.yaml:38) decode with soundfile into float32, average to mono and pad into a
 * (B, N) batch.  This library replaces the soundfile decode + collate with native code:
 *
 *   - FLAC (all subframe kinds: CONSTANT / VERBATIM / FIXED / LPC, Rice and Rice2 residuals with
 *     escapes, independent / left-side / side-right / mid-side stereo, wasted bits, CRC-8 and
 *     CRC-16 verified) and RIFF WAV (PCM u8/s16/s24/s32, IEEE float32/float64, EXTENSIBLE);
 *   - soundfile's float32 scaling (integer sample / 2^(bits-1)) and NeMo AudioSegment's mono
 *     mix (mean over channels);
 *   - a multi-threaded batch loader that decodes B files straight into the rows of a caller-owned
 *     (pinned) (B, row_stride) float32 buffer, zero-padding each row (NeMo _speech_collate_fn).
 *
 * Conventions: plain pointers and sizes; the caller owns all memory; every call returns 0 on
 * success or a negative KDFM_IO_* status, with a thread-local message from kdfm_io_last_error().
 * Calls are re-entrant and hold no global state.
 */
#ifndef KDFM_IO_H
#define KDFM_IO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  KDFM_IO_OK = 0,
  KDFM_IO_ERR_OPEN = -1,      /* file cannot be opened / read */
  KDFM_IO_ERR_FORMAT = -2,    /* not a FLAC / RIFF-WAV stream, or an unsupported encoding */
  KDFM_IO_ERR_CORRUPT = -3,   /* bitstream error or CRC mismatch */
  KDFM_IO_ERR_ARG = -4,       /* bad argument (null pointer, negative size, buffer too small) */
};

/* Stream properties without decoding the samples (soundfile.info, used by the reference to
 * compute manifest durations, asr_train_diffm_GS.py:85-87). */
int kdfm_audio_probe(const char* path, int32_t* sample_rate, int32_t* channels,
                     int32_t* bits_per_sample, int64_t* frames);

/* Decode frames [offset, offset + max_frames) of one file (max_frames < 0: to the end), mixed to
 * mono float32, into out[0 .. *n_out).  `capacity` is the size of `out` in floats.  NeMo
 * AudioSegment.from_file(offset, duration) semantics (offset/duration given here in frames). */
int kdfm_audio_decode(const char* path, int64_t offset, int64_t max_frames, float* out,
                      int64_t capacity, int64_t* n_out, int32_t* sample_rate);

/* Collate: decode n files concurrently on `threads` host threads into the rows of
 * out (n, row_stride) float32; row i receives file i's mono samples [offsets[i], +max_frames[i])
 * (offsets / max_frames may be NULL: whole file), zero-padded to row_stride; lens[i] = samples
 * written.  Rows longer than row_stride are an error (KDFM_IO_ERR_ARG) — size the batch with
 * kdfm_audio_probe first.  expected_rate > 0 rejects files at another sample rate (the reference
 * always trains at 16 kHz, asr_train_diffm.py:1443). */
int kdfm_audio_load_batch(const char* const* paths, int32_t n, const int64_t* offsets,
                          const int64_t* max_frames, float* out, int64_t row_stride, int64_t* lens,
                          int32_t expected_rate, int32_t threads);

const char* kdfm_io_last_error(void);
const char* kdfm_io_version(void);

#ifdef __cplusplus
}
#endif

#endif /* KDFM_IO_H */
