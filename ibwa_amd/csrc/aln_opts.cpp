// aln_opts.cpp -- the `aln` command line (bwa_aln, bwtaln.c:243-328) parsed into gap_opt_t.
// Shared by the CLI (aln_main.cpp) and every other caller of the library (bench.py), so that
// the product configures itself with its own parser.
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "ibwa_aln.h"

namespace {
std::mutex g_getopt_lock;  // getopt keeps global state
}

extern "C" int ibwa_aln_parse_args(int argc, char *const *argv, ibwa_gap_opt_t *opt, int *n_gpus, const char **fn_out) {
  std::lock_guard<std::mutex> lk(g_getopt_lock);
  ibwa_gap_init_opt(opt);  // gap_init_opt (bwtaln.c:21-37)
  if (n_gpus) *n_gpus = 1;
  if (fn_out) *fn_out = nullptr;
  int opte = -1, c;
  optind = 0;  // full re-initialisation (GNU getopt), so the parser can be called again
  opterr = 1;
  // bwtaln.c:249-284, plus -G (number of GPUs)
  while ((c = getopt(argc, argv, "n:o:e:i:d:l:k:cLR:m:t:NM:O:E:q:f:b012IB:G:")) >= 0) {
    switch (c) {
      case 'n':
        if (strstr(optarg, ".")) opt->fnr = (float)atof(optarg), opt->max_diff = -1;
        else opt->max_diff = atoi(optarg), opt->fnr = -1.0f;
        break;
      case 'o': opt->max_gapo = atoi(optarg); break;
      case 'e': opte = atoi(optarg); break;
      case 'M': opt->s_mm = atoi(optarg); break;
      case 'O': opt->s_gapo = atoi(optarg); break;
      case 'E': opt->s_gape = atoi(optarg); break;
      case 'd': opt->max_del_occ = atoi(optarg); break;
      case 'i': opt->indel_end_skip = atoi(optarg); break;
      case 'l': opt->seed_len = atoi(optarg); break;
      case 'k': opt->max_seed_diff = atoi(optarg); break;
      case 'm': opt->max_entries = atoi(optarg); break;
      case 't': opt->n_threads = atoi(optarg); break;
      case 'L': opt->mode |= IBWA_MODE_LOGGAP; break;
      case 'R': opt->max_top2 = atoi(optarg); break;
      case 'q': opt->trim_qual = atoi(optarg); break;
      case 'c': opt->mode &= ~IBWA_MODE_COMPREAD; break;
      case 'N': opt->mode |= IBWA_MODE_NONSTOP; opt->max_top2 = 0x7fffffff; break;
      case 'f': if (fn_out) *fn_out = optarg; break;
      case 'b': opt->mode |= IBWA_MODE_BAM; break;
      case '0': opt->mode |= IBWA_MODE_BAM_SE; break;
      case '1': opt->mode |= IBWA_MODE_BAM_READ1; break;
      case '2': opt->mode |= IBWA_MODE_BAM_READ2; break;
      case 'I': opt->mode |= IBWA_MODE_IL13; break;
      case 'B': opt->mode |= atoi(optarg) << 24; break;
      case 'G': if (n_gpus) *n_gpus = atoi(optarg); break;
      default: return -1;
    }
  }
  if (opte > 0) {  // bwtaln.c:281-284
    opt->max_gape = opte;
    opt->mode &= ~IBWA_MODE_GAPE;
  }
  return optind;
}
