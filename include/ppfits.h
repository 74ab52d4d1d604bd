/* ppfits.h -- native PSRFITS reader for the drop-in's load_data
 * (replaces PSRCHIVE's Archive_load in
 * pplib.load_data, pplib.py:2650-2820, for fold-mode PSRFITS archives).
 *
 * Host-only C ABI (libppfits.so, plain C++): it parses the FITS primary
 * header, the SUBINT binary table and, when present, the POLYCO and HISTORY
 * tables, and hands back the metadata and the raw DATA column in native byte
 * order.  The integer -> physical unpacking (DATA * DAT_SCL + DAT_OFFS) and
 * the polarisation sum run on the GPU (ppf_unpack_subints in ppfit.h), so
 * only the raw 8/16-bit samples cross PCIe.
 *
 * Every function returns 0 or a negative PPFITS_ERR_*; ppfits_error() holds
 * the reason.  Strings are NUL-terminated copies of the header values.
 */
#ifndef PPFITS_H
#define PPFITS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PPFITS_OK 0
#define PPFITS_ERR_IO -1       /* open / read failure                      */
#define PPFITS_ERR_FORMAT -2   /* not FITS, or a malformed header / table  */
#define PPFITS_ERR_MISSING -3  /* a required HDU, keyword or column absent */
#define PPFITS_ERR_RANGE -4    /* subint range outside the table           */

/* raw sample type of the DATA column (its TFORM letter) */
#define PPFITS_RAW_U8 1   /* 'B' */
#define PPFITS_RAW_I16 2  /* 'I' */
#define PPFITS_RAW_F32 3  /* 'E' */

typedef struct ppfits_file ppfits_file;

typedef struct {
  int32_t nsub, npol, nchan, nbin;
  int32_t raw_type;          /* PPFITS_RAW_*                                   */
  int32_t has_period;        /* SUBINT has a PERIOD column                     */
  int32_t has_par_ang;       /* SUBINT has a PAR_ANG column                    */
  int32_t npolyco;           /* rows of the POLYCO table (0: none)             */
  int32_t ncoef;             /* coefficients per POLYCO row                    */
  int32_t dedispersed;       /* last HISTORY row's DEDISP (0 if no HISTORY)    */
  int32_t stt_imjd;          /* start MJD, integer day                         */
  double stt_smjd, stt_offs; /* start seconds of day, fractional seconds      */
  double obsfreq, obsbw;     /* centre frequency, bandwidth [MHz]              */
  double chan_dm;            /* primary CHAN_DM (NaN if absent)                */
  double dm;                 /* SUBINT DM (NaN if absent)                      */
  double be_delay;           /* primary BE_DELAY [s] (0 if absent)             */
  double chan_bw;            /* SUBINT CHAN_BW [MHz] (NaN if absent)           */
  char telescope[32], frontend[32], backend[32], source[32];
  char pol_type[16], obs_mode[16];
} ppfits_info;

int ppfits_open(const char* path, ppfits_file** out);
void ppfits_close(ppfits_file* f);
const char* ppfits_error(const ppfits_file* f);
int ppfits_get_info(const ppfits_file* f, ppfits_info* out);

/* Per-subint metadata, C order (any pointer may be NULL):
 *   freqs [nsub][nchan] (DAT_FREQ), wts [nsub][nchan] (DAT_WTS),
 *   offs, scl [nsub][npol][nchan] (DAT_OFFS, DAT_SCL),
 *   tsubint, offs_sub, period, par_ang [nsub] (NaN where a column is absent) */
int ppfits_read_meta(const ppfits_file* f, double* freqs, double* wts, double* offs,
                     double* scl, double* tsubint, double* offs_sub, double* period,
                     double* par_ang);

/* Raw DATA of subints [isub0, isub0 + n) in native byte order, C order
 * [n][npol][nchan][nbin] of the raw type (1, 2 or 4 bytes per sample).    */
int ppfits_read_raw(const ppfits_file* f, int32_t isub0, int32_t n, void* out);

/* POLYCO rows (tempo polynomial predictors): ref_mjd, ref_f0, ref_phs,
 * nspan [min] per row and coeff [npolyco][ncoef].                          */
int ppfits_read_polyco(const ppfits_file* f, double* ref_mjd, double* ref_f0, double* ref_phs,
                       double* nspan, double* coeff);

#ifdef __cplusplus
}
#endif

#endif /* PPFITS_H */
