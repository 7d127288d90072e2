// pqwriter.cpp — host-side page WRITER used to synthesize parquet-mr-identical
// pages for the benchmark workloads and the tests (libpqwriter.so).
//
// parquet-mr's writers are out of scope as a product; they are
// restated here only so that synthetic inputs are byte-identical to what
// parquet-mr 1.15 would emit for the same values:
//   RunLengthBitPackingHybridEncoder   parquet-column/.../rle/RunLengthBitPackingHybridEncoder.java:146-273
//   DeltaBinaryPackingValuesWriterForLong / ForInteger
//                                      parquet-column/.../delta/DeltaBinaryPackingValuesWriterForLong.java:75-185
//                                      parquet-column/.../delta/DeltaBinaryPackingValuesWriterForInteger.java:75-185
//   BytesUtils.writeUnsignedVarInt / writeZigZagVarLong / writeIntLittleEndianPaddedOnBitWidth
//                                      parquet-common/.../bytes/BytesUtils.java:150-290
//   pack8Values (LSB first)            ByteBasedBitPackingGenerator.generatePack :214-246
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <limits>
#include <type_traits>
#include <vector>

namespace {

struct Out {
  std::vector<uint8_t> b;
  void put(uint8_t x) { b.push_back(x); }
  void put(const uint8_t* p, size_t n) { b.insert(b.end(), p, p + n); }
};

void write_uvarint(uint32_t v, Out& o) {  // writeUnsignedVarInt(int) :185-191
  while ((v & 0xFFFFFF80u) != 0) {
    o.put(uint8_t((v & 0x7F) | 0x80));
    v >>= 7;
  }
  o.put(uint8_t(v & 0x7F));
}

void write_uvarlong(uint64_t v, Out& o) {  // writeUnsignedVarLong :271-277
  while ((v & 0xFFFFFFFFFFFFFF80ull) != 0) {
    o.put(uint8_t((v & 0x7F) | 0x80));
    v >>= 7;
  }
  o.put(uint8_t(v & 0x7F));
}

void write_zigzag_varlong(int64_t v, Out& o) {  // writeZigZagVarLong :287-289
  write_uvarlong((uint64_t(v) << 1) ^ uint64_t(v >> 63), o);
}

void write_zigzag_varint(int32_t v, Out& o) {  // writeZigZagVarInt :201-203
  write_uvarint((uint32_t(v) << 1) ^ uint32_t(v >> 31), o);
}

void write_int_le_padded(Out& o, int32_t v, int bit_width) {  // :162-182
  int bytes = (bit_width + 7) / 8;
  for (int i = 0; i < bytes; i++) o.put(uint8_t((uint32_t(v) >> (8 * i)) & 0xFF));
}

// pack8Values, LSB first: value i -> bits [i*w, (i+1)*w), masked to w bits.
template <typename T>
void pack8(const T* in, int w, uint8_t* out) {
  std::memset(out, 0, size_t(w));
  if (w == 0) return;
  for (int i = 0; i < 8; i++) {
    uint64_t v = uint64_t(in[i]);
    if (w < 64) v &= (uint64_t(1) << w) - 1;
    for (int k = 0; k < w; k++) {
      int bit = i * w + k;
      if ((v >> k) & 1) out[bit >> 3] |= uint8_t(1u << (bit & 7));
    }
  }
}

// RunLengthBitPackingHybridEncoder (the <encoded-data> part of the grammar, :32-57)
class RleEncoder {
 public:
  explicit RleEncoder(int bit_width) : w_(bit_width) { pack_buf_.resize(size_t(w_ > 0 ? w_ : 1)); }

  void write_int(int32_t value) {  // writeInt :146-189
    if (value == previous_) {
      ++repeat_;
      if (repeat_ >= 8) return;
    } else {
      if (repeat_ >= 8) write_rle_run();
      repeat_ = 1;
      previous_ = value;
    }
    buffered_[nbuf_++] = value;
    if (nbuf_ == 8) write_or_append_bit_packed_run();
  }

  std::vector<uint8_t> to_bytes() {  // toBytes :253-273
    if (repeat_ >= 8) {
      write_rle_run();
    } else if (nbuf_ > 0) {
      for (int i = nbuf_; i < 8; i++) buffered_[i] = 0;
      write_or_append_bit_packed_run();
      end_previous_bit_packed_run();
    } else {
      end_previous_bit_packed_run();
    }
    return o_.b;
  }

 private:
  void write_or_append_bit_packed_run() {  // :191-219
    if (groups_ >= 63) end_previous_bit_packed_run();
    if (header_ptr_ == -1) {
      o_.put(0);  // sentinel
      header_ptr_ = int64_t(o_.b.size()) - 1;
    }
    pack8(buffered_, w_, pack_buf_.data());
    o_.put(pack_buf_.data(), size_t(w_));
    nbuf_ = 0;
    repeat_ = 0;
    ++groups_;
  }

  void end_previous_bit_packed_run() {  // :228-245
    if (header_ptr_ == -1) return;
    o_.b[size_t(header_ptr_)] = uint8_t((groups_ << 1) | 1);
    header_ptr_ = -1;
    groups_ = 0;
  }

  void write_rle_run() {  // :247-264
    end_previous_bit_packed_run();
    write_uvarint(uint32_t(repeat_) << 1, o_);
    write_int_le_padded(o_, previous_, w_);
    repeat_ = 0;
    nbuf_ = 0;
  }

  int w_;
  Out o_;
  std::vector<uint8_t> pack_buf_;
  int32_t previous_ = 0;
  int32_t buffered_[8] = {0};
  int nbuf_ = 0;
  int32_t repeat_ = 0;
  int groups_ = 0;
  int64_t header_ptr_ = -1;
};

// DeltaBinaryPackingValuesWriterForLong / ForInteger. T = int64_t or int32_t;
// deltas wrap in T (Java long / int ring). Stale bit widths and stale
// deltaBlockBuffer entries past the last value are reproduced (:101-137).
template <typename T>
class DeltaEncoder {
 public:
  DeltaEncoder(int block, int mb_num) : block_(block), mb_num_(mb_num), mb_size_(block / mb_num) {
    delta_.assign(size_t(block_), 0);
    widths_.assign(size_t(mb_num_), 0);
  }

  void write(T v) {  // writeLong :75-99 / writeInteger
    total_++;
    if (total_ == 1) {
      first_ = v;
      prev_ = v;
      return;
    }
    using U = typename std::make_unsigned<T>::type;
    T d = T(U(v) - U(prev_));
    prev_ = v;
    delta_[size_t(to_flush_++)] = d;
    if (d < min_delta_) min_delta_ = d;
    if (to_flush_ == block_) flush();
  }

  std::vector<uint8_t> get_bytes() {  // getBytes :174-185
    if (to_flush_ != 0) flush();
    Out h;
    write_uvarint(uint32_t(block_), h);
    write_uvarint(uint32_t(mb_num_), h);
    write_uvarint(uint32_t(total_), h);
    if (sizeof(T) == 8)
      write_zigzag_varlong(int64_t(first_), h);  // BytesInput.fromZigZagVarLong (ForLong :182)
    else
      write_zigzag_varint(int32_t(first_), h);   // BytesInput.fromZigZagVarInt (ForInteger :178)
    h.put(o_.b.data(), o_.b.size());
    return h.b;
  }

 private:
  void flush() {  // flushBlockBuffer :101-137
    using U = typename std::make_unsigned<T>::type;
    for (int i = 0; i < to_flush_; i++) delta_[size_t(i)] = T(U(delta_[size_t(i)]) - U(min_delta_));
    if (sizeof(T) == 8)
      write_zigzag_varlong(int64_t(min_delta_), o_);
    else
      write_zigzag_varint(int32_t(min_delta_), o_);
    int mbs = (to_flush_ + mb_size_ - 1) / mb_size_;  // getMiniBlockCountToFlush
    for (int m = 0; m < mbs; m++) {  // calculateBitWidthsForDeltaBlockBuffer :147-163
      U mask = 0;
      int s = m * mb_size_, e = std::min((m + 1) * mb_size_, to_flush_);
      for (int i = s; i < e; i++) mask |= U(delta_[size_t(i)]);
      int w = 0;
      while (mask) { w++; mask >>= 1; }
      widths_[size_t(m)] = w;
    }
    for (int m = 0; m < mb_num_; m++) o_.put(uint8_t(widths_[size_t(m)]));
    uint8_t buf[64];
    for (int m = 0; m < mbs; m++) {
      int w = widths_[size_t(m)];
      for (int j = m * mb_size_; j < (m + 1) * mb_size_; j += 8) {
        pack8(&delta_[size_t(j)], w, buf);
        o_.put(buf, size_t(w));
      }
    }
    min_delta_ = std::numeric_limits<T>::max();
    to_flush_ = 0;
  }

  int block_, mb_num_, mb_size_;
  std::vector<T> delta_;
  std::vector<int> widths_;
  int32_t total_ = 0;
  int to_flush_ = 0;
  T first_ = 0, prev_ = 0;
  T min_delta_ = std::numeric_limits<T>::max();
  Out o_;
};

int64_t copy_out(const std::vector<uint8_t>& b, uint8_t* out, int64_t cap) {
  if (int64_t(b.size()) > cap) return -int64_t(b.size());
  if (!b.empty()) std::memcpy(out, b.data(), b.size());
  return int64_t(b.size());
}

}  // namespace

extern "C" {

// Encoded <encoded-data> of the RLE/bit-packed hybrid for n values. Returns the
// byte count, or -(needed) when cap is too small.
int64_t pqw_rle_encode(int bit_width, const int32_t* values, int64_t n, uint8_t* out, int64_t cap) {
  if (bit_width < 0 || bit_width > 32) return 0;
  RleEncoder enc(bit_width);
  for (int64_t i = 0; i < n; i++) enc.write_int(values[i]);
  return copy_out(enc.to_bytes(), out, cap);
}

// Same, for uint8 inputs (definition / repetition levels).
int64_t pqw_rle_encode_u8(int bit_width, const uint8_t* values, int64_t n, uint8_t* out, int64_t cap) {
  if (bit_width < 0 || bit_width > 32) return 0;
  RleEncoder enc(bit_width);
  for (int64_t i = 0; i < n; i++) enc.write_int(values[i]);
  return copy_out(enc.to_bytes(), out, cap);
}

int64_t pqw_delta_encode_long(const int64_t* values, int64_t n, int block, int mb_num, uint8_t* out, int64_t cap) {
  if (mb_num <= 0 || block % mb_num != 0 || (block / mb_num) % 8 != 0) return 0;
  DeltaEncoder<int64_t> enc(block, mb_num);
  for (int64_t i = 0; i < n; i++) enc.write(values[i]);
  return copy_out(enc.get_bytes(), out, cap);
}

int64_t pqw_delta_encode_int(const int32_t* values, int64_t n, int block, int mb_num, uint8_t* out, int64_t cap) {
  if (mb_num <= 0 || block % mb_num != 0 || (block / mb_num) % 8 != 0) return 0;
  DeltaEncoder<int32_t> enc(block, mb_num);
  for (int64_t i = 0; i < n; i++) enc.write(values[i]);
  return copy_out(enc.get_bytes(), out, cap);
}

// pack8Values (LSB first) for w in [0, 64]: 8 values -> w bytes.
void pqw_pack8_long(const int64_t* in, int w, uint8_t* out) { pack8(in, w, out); }

}  // extern "C"
