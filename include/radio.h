/* radio.h — C ABI of libradio.so: native FLAC reading for the data path (host code, no GPU).
 *
 * Replaces the reference's per-utterance `soundfile.read(str(base_dir / f"flac/{key}.flac"))`
 * (src/data_utils.py:165 Dataset_ASVspoof2019_train, :200 Dataset_ASVspoof2019_devNeval,
 * :221 Dataset_ASVspoof2021_eval). Values are libsndfile's float normalisation, x / 2^(bits-1).
 *
 * Conventions: return 0 on success, a negative RDX_IO_* code otherwise (rdx_io_strerror names it);
 * caller-owned buffers; no global state; every call is thread-safe.
 */
#ifndef RADIO_H
#define RADIO_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum {
  RDX_IO_ENOENT = -101,    /* file cannot be opened/read */
  RDX_IO_EFORMAT = -102,   /* no fLaC marker or STREAMINFO */
  RDX_IO_ECORRUPT = -103,  /* bad frame header, subframe, CRC-8/CRC-16, or sample count != STREAMINFO */
  RDX_IO_ESHORT = -104,    /* decoded more frames than the capacity given (frames_out holds the count) */
  RDX_IO_ECHANNELS = -105, /* batch loader: file is not mono */
  RDX_IO_EARG = -106
};

const char* rdx_io_strerror(int code);

/* STREAMINFO of a file: frames per channel (0 if the encoder left it unknown), channels, rate, bits. */
int rdx_flac_probe(const char* path, int64_t* frames, int* channels, int* sample_rate, int* bits);

/* Decode a whole file / in-memory stream to interleaved float64 [frames, channels]
 * (soundfile.read(path) -> float64 array; the reference's sf.read default). */
int rdx_flac_read(const char* path, double* out, int64_t cap_frames, int64_t* frames_out);
int rdx_flac_decode_mem(const uint8_t* data, int64_t nbytes, double* out, int64_t cap_frames,
                        int64_t* frames_out, int* channels, int* sample_rate);

/* Batch loader: decode n mono files with `threads` host threads into one float32 buffer,
 * file i at out + offsets[i] with room for caps[i] samples. frames_out[i] / status[i] per file;
 * the return value is the first failing status (0 if all succeeded). */
int rdx_flac_read_batch(const char* const* paths, int n, float* out, const int64_t* offsets,
                        const int64_t* caps, int64_t* frames_out, int* status, int threads);

#ifdef __cplusplus
}
#endif
#endif
