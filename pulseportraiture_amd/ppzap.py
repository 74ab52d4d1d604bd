"""ppzap drop-in: flag bad channels (ppzap.py:18-95).

Two algorithms, as in the reference:
- ``GetTOAs.get_channels_to_zap`` (pptoas.py:1201-1278) after ``get_TOAs``:
  per-channel reduced chi2 of the fitted portrait (one fused device call per
  archive, ppf_resid_chi2_rows) plus the iterated S/N cut;
- ``get_zap_channels`` (ppzap.py:18-48): the iterated median + nstd * std cut
  on the channel noise levels -- nchan numbers per subint, host arithmetic.

``print_paz_cmds`` writes the PSRCHIVE ``paz`` commands (ppzap.py:50-95).
The command-line front end is out of scope.
"""
import sys

import numpy as np


def get_zap_channels(data, nstd=3):
    """Channels whose noise is more than nstd standard deviations above the
    subint median, removed and re-tested until none is flagged
    (ppzap.py:18-48).  ``data`` needs ok_isubs, ok_ichans and noise_stds."""
    zap_channels = []
    noise_stds = np.asarray(data.noise_stds)
    for isub in data.ok_isubs:
        ichans = list(np.copy(data.ok_ichans[isub]))
        zap_ichans = []
        while len(ichans):
            ns = noise_stds[isub, 0, ichans]
            median = np.median(ns)
            std = np.std(ns)
            bad = list(np.where(ns > median + nstd * std)[0])
            if not len(bad):
                break
            flagged = list(np.array(ichans)[bad])
            zap_ichans.extend(flagged)
            for ichan in flagged:
                ichans.pop(ichans.index(ichan))
        zap_ichans.sort()
        zap_channels.append(zap_ichans)
    return zap_channels


def print_paz_cmds(datafiles, zap_list, all_subs=False, modify=True, outfile=None,
                   quiet=False):
    """Print (or append to outfile) the paz commands that zap zap_list[iarch][isub]
    (ppzap.py:50-95).  Returns the lines written."""
    if not len(datafiles) or not len(zap_list):
        if not quiet:
            print("Nothing to zap.")
            return None
    lines = []
    paz_outfile = None
    for iarch, datafile in enumerate(datafiles):
        count = sum(len(z) for z in zap_list[iarch])
        if count:
            if modify:
                paz_outfile = datafile
            else:
                ii = datafile[::-1].find(".")
                paz_outfile = datafile + ".zap" if ii < 0 else datafile[:-ii] + "zap"
                lines.append("paz -e zap %s" % datafile)
        last_line = ""
        for isub, bad_ichans in enumerate(zap_list[iarch]):
            for bad_ichan in bad_ichans:
                if not all_subs:
                    lines.append("paz -m -I -z %d -w %d %s" % (bad_ichan, isub, paz_outfile))
                else:
                    line = "paz -m -z %d %s" % (bad_ichan, paz_outfile)
                    if line != last_line:
                        lines.append(line)
                    last_line = line
    out = open(outfile, "a") if outfile is not None else sys.stdout
    try:
        for line in lines:
            out.write(line + "\n")
    finally:
        if outfile is not None:
            out.close()
    if outfile is not None and not quiet:
        print("Wrote %s." % outfile)
    return lines
