// `lda` CLI -- the oni-lda-c command-line contract ([U-H]):
//
//   lda est <alpha> <k> <settings> [nproc] <data> <random|seeded|model-prefix> <directory>
//   lda inf <settings> <model-prefix> <data> <name>
//
// oni-ml invoked `mpiexec -n P ./lda est 2.5 20 settings.txt P model.dat random dir`; the optional
// [nproc] argument is accepted here and mapped to OpenMP threads (no MPI on a single node).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <sys/stat.h>

#include "lda_vem.h"

static int usage() {
  std::fprintf(stderr,
               "usage: lda est <alpha> <k> <settings> [nproc] <data> <random|seeded|*> <directory>\n"
               "       lda inf <settings> <model> <data> <name>\n");
  return 2;
}

int main(int argc, char** argv) {
  if (argc < 2) return usage();
  const std::string cmd = argv[1];
  std::string err;
  oni_lda::Settings s;
  if (cmd == "est") {
    if (argc != 8 && argc != 9) return usage();
    const double alpha = std::atof(argv[2]);
    const int K = std::atoi(argv[3]);
    if (!oni_lda::read_settings(argv[4], &s, &err)) {
      std::fprintf(stderr, "lda: %s\n", err.c_str());
      return 1;
    }
    int a = 5;
    if (argc == 9) s.threads = std::atoi(argv[a++]);
    const std::string data = argv[a++], init = argv[a++], dir = argv[a++];
    mkdir(dir.c_str(), 0755);
    oni_lda::Corpus c;
    if (!oni_lda::read_corpus(data, &c, &err)) {
      std::fprintf(stderr, "lda: %s\n", err.c_str());
      return 1;
    }
    std::fprintf(stderr, "lda est: %d docs, %d terms, K=%d\n", c.num_docs(), c.num_terms, K);
    oni_lda::Model m;
    auto r = oni_lda::run_em(c, &m, K, alpha, init, s, dir);
    if (r.iterations == 0) return 1;
    std::fprintf(stderr, "lda est: %d EM iterations, final likelihood %.6f, alpha %.6f\n", r.iterations,
                 r.likelihood.empty() ? 0.0 : r.likelihood.back(), m.alpha);
    return 0;
  }
  if (cmd == "inf") {
    if (argc != 6) return usage();
    if (!oni_lda::read_settings(argv[2], &s, &err)) {
      std::fprintf(stderr, "lda: %s\n", err.c_str());
      return 1;
    }
    oni_lda::Model m;
    if (!oni_lda::load_model(argv[3], &m, &err)) {
      std::fprintf(stderr, "lda: %s\n", err.c_str());
      return 1;
    }
    oni_lda::Corpus c;
    if (!oni_lda::read_corpus(argv[4], &c, &err)) {
      std::fprintf(stderr, "lda: %s\n", err.c_str());
      return 1;
    }
    std::vector<double> gamma;
    auto lik = oni_lda::infer(c, m, s, &gamma);
    const std::string name = argv[5];
    oni_lda::save_gamma(gamma, c.num_docs(), m.K, name + "-gamma.dat");
    FILE* f = std::fopen((name + "-lda-lhood.dat").c_str(), "w");
    if (f) {
      for (double l : lik) std::fprintf(f, "%5.5f\n", l);
      std::fclose(f);
    }
    return 0;
  }
  return usage();
}
