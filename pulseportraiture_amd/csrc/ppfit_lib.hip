// ppfit_lib.hip -- single translation unit for libppfit.so (gfx950).
#include "ppfit_spectra.hip"
#include "ppfit_fit.hip"
#include "ppfit_taylor.hip"
#include "ppfit_tnc.hip"
#include "ppfit_ncg.hip"
#include "ppfit_models.hip"
#include "ppfit_generic.hip"
#include "ppfit_capi.hip"
