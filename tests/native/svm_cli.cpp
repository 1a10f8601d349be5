// Command-line face of the svmlight parser (krcn_svmlight.hip) for the host
// sanitizer builds: tests/test_sanitizers.py parses the inputs of
// tests/test_libsvm.py through it and compares with sklearn.
//   svm_cli <file> <threads> <out.bin>
// out.bin: int64 rows, nnz, max index, min index; int64 indptr[rows + 1],
// int64 indices[nnz] (unshifted), float64 data[nnz], float64 labels[rows].
// A parse error prints the library's message on stderr and exits 2.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <vector>

#include "krcn_host.hpp"

int main(int argc, char** argv) {
  if (argc != 4) {
    std::fprintf(stderr, "usage: svm_cli <file> <threads> <out.bin>\n");
    return 1;
  }
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> text((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  krcn_svm* p = nullptr;
  int64_t info[4];
  if (krcn_svm_parse(text.data(), int64_t(text.size()), std::atoi(argv[2]), &p, info) != KRCN_OK) {
    std::fprintf(stderr, "%s\n", krcn_last_error_string());
    return 2;
  }
  const int64_t rows = info[0], nnz = info[1];
  std::vector<int32_t> ip(size_t(rows) + 1), ix(size_t(nnz) + 1);
  std::vector<double> dv(size_t(nnz) + 1), lb(size_t(rows) + 1);
  if (krcn_svm_export(p, 0, ip.data(), ix.data(), dv.data(), lb.data()) != KRCN_OK) {
    std::fprintf(stderr, "%s\n", krcn_last_error_string());
    return 3;
  }
  std::vector<int64_t> ip64(ip.begin(), ip.end()), ix64(ix.begin(), ix.begin() + nnz);
  std::FILE* o = std::fopen(argv[3], "wb");
  std::fwrite(info, sizeof(int64_t), 4, o);
  std::fwrite(ip64.data(), sizeof(int64_t), size_t(rows) + 1, o);
  std::fwrite(ix64.data(), sizeof(int64_t), size_t(nnz), o);
  std::fwrite(dv.data(), sizeof(double), size_t(nnz), o);
  std::fwrite(lb.data(), sizeof(double), size_t(rows), o);
  std::fclose(o);
  krcn_svm_destroy(p);
  return 0;
}
