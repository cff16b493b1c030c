// Driver of the emulated Zstd compressor kernel (tools/simt_emu/emu_build.sh).
//   zstdc_emu IN.bin LENS.u32 LEVEL MAX_LEN OUT.bin OUTLENS.u32
// Compresses the blocks (lengths in LENS, packed in IN) one emulated
// workgroup at a time; writes the frames packed, their lengths and statuses.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

namespace lvkv {
hipError_t launch_zstd_compress(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                uint8_t* dst, const uint64_t* dst_off, uint32_t* dst_len,
                                uint8_t* status, uint32_t nblocks, uint32_t max_len, int level,
                                uint64_t dst_stride, hipStream_t stream);
}

static std::vector<uint8_t> slurp(const char* p) {
  FILE* f = fopen(p, "rb");
  if (!f) exit(2);
  fseek(f, 0, SEEK_END);
  std::vector<uint8_t> v(ftell(f));
  fseek(f, 0, SEEK_SET);
  if (fread(v.data(), 1, v.size(), f) != v.size()) exit(2);
  fclose(f);
  return v;
}

int main(int argc, char** argv) {
  if (argc != 7) return 2;
  std::vector<uint8_t> in = slurp(argv[1]), lb = slurp(argv[2]);
  const uint32_t n = lb.size() / 4;
  const int level = atoi(argv[3]);
  const uint32_t max_len = strtoul(argv[4], 0, 10);
  std::vector<uint32_t> len(n);
  memcpy(len.data(), lb.data(), 4 * n);
  std::vector<uint64_t> off(n), doff(n);
  uint64_t p = 0, q = 0;
  for (uint32_t i = 0; i < n; ++i) {
    off[i] = p;
    doff[i] = q;
    p += len[i];
    q += len[i] + (len[i] >> 8) + (len[i] < 131072 ? (131072 - len[i]) >> 11 : 0) + 16;
  }
  in.resize(p + 64);
  std::vector<uint8_t> dst(q + 64), st(n);
  std::vector<uint32_t> dl(n);
  lvkv::launch_zstd_compress(in.data(), off.data(), len.data(), dst.data(), doff.data(), dl.data(),
                             st.data(), n, max_len, level, 0, nullptr);
  FILE* fo = fopen(argv[5], "wb");
  FILE* fl = fopen(argv[6], "wb");
  for (uint32_t i = 0; i < n; ++i) {
    fwrite(dst.data() + doff[i], 1, dl[i], fo);
    const uint32_t rec[2] = {dl[i], st[i]};
    fwrite(rec, 4, 2, fl);
  }
  fclose(fo);
  fclose(fl);
  return 0;
}
