// hrs.hpp — header-only C++17 mirror of the hops codec plugin interface over
// the C ABI in hrs.h, for native callers (the C++ analogue of the JNI shim).
//
//   hrs::ErasureCode        io.hops.erasure_coding.ErasureCode
//                           (hadoop-hdfs/.../io/hops/erasure_coding/ErasureCode.java:25-182)
//   hrs::HipReedSolomonCode ReedSolomonCode (hops-erasure-coding/.../ReedSolomonCode.java)
//   hrs::HipXORCode         XORCode        (hops-erasure-coding/.../XORCode.java)
//   hrs::IOException / hrs::TooManyErasedLocations  the Java exceptions
//
// Java's byte[][] rows carry their length; here rows are raw pointers plus one
// `len` for the call, as Encoder.java:442 / Decoder.java:352 pass equal-length rows.
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "hrs.h"

namespace hrs {

class IOException : public std::runtime_error {
 public:
  explicit IOException(const std::string& m, int status = HRS_EDEVICE) : std::runtime_error(m), status_(status) {}
  int status() const { return status_; }

 private:
  int status_;
};

// TooManyErasedLocations extends IOException (TooManyErasedLocations.java:26-31).
class TooManyErasedLocations : public IOException {
 public:
  explicit TooManyErasedLocations(const std::string& m) : IOException(m, HRS_ETOOMANY) {}
};

inline void check(hrs_status st, const hrs_codec* c) {
  if (st == HRS_OK) return;
  const std::string msg = hrs_last_error(c);
  if (st == HRS_ETOOMANY) throw TooManyErasedLocations(msg);
  if (st == HRS_EINVAL) throw std::invalid_argument(msg);
  throw IOException(msg, st);
}

class ErasureCode {
 public:
  virtual ~ErasureCode() = default;
  virtual int stripeSize() const = 0;
  virtual int paritySize() const = 0;
  virtual int symbolSize() const = 0;
  // ErasureCode.java:136-156 / :162-181
  virtual void encodeBulk(const std::vector<uint8_t*>& inputs, const std::vector<uint8_t*>& outputs,
                          size_t len) = 0;
  virtual void decodeBulk(const std::vector<uint8_t*>& readBufs, const std::vector<uint8_t*>& writeBufs,
                          size_t len, const std::vector<int>& erasedLocations,
                          const std::vector<int>& locationsToRead,
                          const std::vector<int>& locationsNotToRead) = 0;
  // ErasureCode.java:89-113 — the k highest-index locations not erased, highest first.
  virtual std::vector<int> locationsToReadForDecode(const std::vector<int>& erasedLocations) const {
    std::vector<int> out;
    const int limit = stripeSize() + paritySize();
    for (int loc = limit - 1; loc >= 0; --loc) {
      bool erased = false;
      for (int e : erasedLocations) erased |= e == loc;
      if (!erased) {
        out.push_back(loc);
        if (static_cast<int>(out.size()) == stripeSize()) break;
      }
    }
    if (static_cast<int>(out.size()) != stripeSize()) {
      std::string s = "Locations ";
      for (int e : erasedLocations) s += " " + std::to_string(e);
      throw TooManyErasedLocations(s);
    }
    return out;
  }
};

// Common owner of an hrs_codec handle.
class HipCode : public ErasureCode {
 public:
  HipCode(int code, int k, int p, int device = -1, int srcParities = 0) {
    hrs_opts o{};
    o.device = device;
    hrs_codec* c = nullptr;
    hrs_status st = code == HRS_CODE_SRC ? hrs_create_src(k, p, srcParities, &o, &c) : hrs_create_code(code, k, p, &o, &c);
    if (st != HRS_OK) check(st, nullptr);
    h_ = c;
  }
  ~HipCode() override { hrs_destroy(h_); }
  HipCode(const HipCode&) = delete;
  HipCode& operator=(const HipCode&) = delete;

  int stripeSize() const override { return hrs_stripe_size(h_); }
  int paritySize() const override { return hrs_parity_size(h_); }
  int symbolSize() const override { return hrs_symbol_size(h_); }
  hrs_codec* handle() const { return h_; }
  // the GPU this codec runs on (hrs_codec_device; hrs_opts.device at creation)
  int device() const { return hrs_codec_device(h_); }

  // the product's list (hrs_locations_to_read_list): SRC returns a local group
  std::vector<int> locationsToReadForDecode(const std::vector<int>& erasedLocations) const override {
    std::vector<int> out(stripeSize() + paritySize());
    int m = 0;
    check(hrs_locations_to_read_list(h_, erasedLocations.data(), static_cast<int>(erasedLocations.size()), out.data(),
                                     &m),
          h_);
    out.resize(m);
    return out;
  }

  void encodeBulk(const std::vector<uint8_t*>& inputs, const std::vector<uint8_t*>& outputs, size_t len) override {
    if (static_cast<int>(inputs.size()) != stripeSize() || static_cast<int>(outputs.size()) != paritySize())
      throw std::invalid_argument("encodeBulk: row counts do not match the codec");
    std::vector<const uint8_t*> in(inputs.begin(), inputs.end());
    check(hrs_encode(h_, in.data(), outputs.data(), len), h_);
  }

  void decodeBulk(const std::vector<uint8_t*>& readBufs, const std::vector<uint8_t*>& writeBufs, size_t len,
                  const std::vector<int>& erased, const std::vector<int>& toRead,
                  const std::vector<int>& notToRead) override {
    if (static_cast<int>(readBufs.size()) != stripeSize() + paritySize() || writeBufs.size() != erased.size())
      throw std::invalid_argument("decodeBulk: row counts do not match");
    std::vector<const uint8_t*> in(readBufs.begin(), readBufs.end());
    check(hrs_decode(h_, in.data(), writeBufs.data(), erased.data(), static_cast<int>(erased.size()),
                     toRead.data(), static_cast<int>(toRead.size()), notToRead.data(),
                     static_cast<int>(notToRead.size()), len),
          h_);
  }

  // encodeBulk plus Encoder.encodeStripe's block checksums (Encoder.java:408-450):
  // crcs (k + p: sources, then parities) are java.util.zip.CRC32 values
  // continued over this round's cells; start them at 0 for fresh CRC32 objects.
  void encodeBulkCrc(const std::vector<uint8_t*>& inputs, const std::vector<uint8_t*>& outputs, size_t len,
                     std::vector<uint32_t>& crcs) {
    if (static_cast<int>(inputs.size()) != stripeSize() || static_cast<int>(outputs.size()) != paritySize() ||
        static_cast<int>(crcs.size()) != stripeSize() + paritySize())
      throw std::invalid_argument("encodeBulkCrc: row or checksum counts do not match the codec");
    std::vector<const uint8_t*> in(inputs.begin(), inputs.end());
    check(hrs_encode_crc(h_, in.data(), outputs.data(), len, crcs.data(), crcs.data()), h_);
  }

  // decodeBulk plus the CRC32 of each repaired buffer (Decoder.java:222-229,
  // :645-655), continued in crcs (one per erased location).
  void decodeBulkCrc(const std::vector<uint8_t*>& readBufs, const std::vector<uint8_t*>& writeBufs, size_t len,
                     const std::vector<int>& erased, const std::vector<int>& toRead,
                     const std::vector<int>& notToRead, std::vector<uint32_t>& crcs) {
    if (static_cast<int>(readBufs.size()) != stripeSize() + paritySize() || writeBufs.size() != erased.size() ||
        crcs.size() != erased.size())
      throw std::invalid_argument("decodeBulkCrc: row or checksum counts do not match");
    std::vector<const uint8_t*> in(readBufs.begin(), readBufs.end());
    check(hrs_decode_crc(h_, in.data(), writeBufs.data(), erased.data(), static_cast<int>(erased.size()),
                         toRead.data(), static_cast<int>(toRead.size()), notToRead.data(),
                         static_cast<int>(notToRead.size()), len, crcs.data(), crcs.data()),
          h_);
  }

  // Asynchronous rounds (hrs_encode_submit / hrs_decode_submit / hrs_collect):
  // submit returns once the rows are staged; collect waits and copies out.
  // checksums: the operation also computes the block CRC32s; collect then
  // continues the running values in *crcs (k + p for encode, one per erased
  // location for decode).
  uint64_t encodeBulkSubmit(const std::vector<uint8_t*>& inputs, size_t len, bool checksums) {
    if (static_cast<int>(inputs.size()) != stripeSize()) throw std::invalid_argument("encodeBulkSubmit: row count");
    std::vector<const uint8_t*> in(inputs.begin(), inputs.end());
    uint64_t t = 0;
    check(hrs_encode_submit(h_, in.data(), len, checksums ? 1 : 0, &t), h_);
    return t;
  }

  uint64_t decodeBulkSubmit(const std::vector<uint8_t*>& readBufs, size_t len, const std::vector<int>& erased,
                            const std::vector<int>& toRead, const std::vector<int>& notToRead, bool checksums) {
    if (static_cast<int>(readBufs.size()) != stripeSize() + paritySize())
      throw std::invalid_argument("decodeBulkSubmit: row count");
    std::vector<const uint8_t*> in(readBufs.begin(), readBufs.end());
    uint64_t t = 0;
    check(hrs_decode_submit(h_, in.data(), erased.data(), static_cast<int>(erased.size()), toRead.data(),
                            static_cast<int>(toRead.size()), notToRead.data(), static_cast<int>(notToRead.size()),
                            len, checksums ? 1 : 0, &t),
          h_);
    return t;
  }

  // Blocks until the operation's GPU work is done (hrs_wait); collect then
  // only copies.
  void wait(uint64_t ticket) { check(hrs_wait(h_, ticket), h_); }

  // Drop an uncollected operation (its slot is drained and freed).
  void release(uint64_t ticket) { check(hrs_release(h_, ticket), h_); }

  // outputs must hold the operation's output rows exactly, and *crcs (a
  // checksummed operation only) its CRC values: hrs_collect writes that many.
  void collect(uint64_t ticket, const std::vector<uint8_t*>& outputs, std::vector<uint32_t>* crcs) {
    int nout = 0, ncrc = 0;
    size_t len = 0;
    check(hrs_ticket_shape(h_, ticket, &nout, &len, &ncrc), h_);
    if (static_cast<int>(outputs.size()) != nout)
      throw std::invalid_argument("collect: " + std::to_string(outputs.size()) + " output rows, the operation has " +
                                  std::to_string(nout));
    if (ncrc > 0 && (!crcs || static_cast<int>(crcs->size()) != ncrc))
      throw std::invalid_argument("collect: the operation keeps " + std::to_string(ncrc) + " CRC values");
    check(hrs_collect(h_, ticket, outputs.data(), crcs ? crcs->data() : nullptr), h_);
  }

  // RS-specific decodeBulk(readBufs, writeBufs, erasedLocation), ReedSolomonCode.java:168-185.
  void decodeBulk3(const std::vector<uint8_t*>& readBufs, const std::vector<uint8_t*>& writeBufs, size_t len,
                   const std::vector<int>& erased) {
    std::vector<const uint8_t*> in(readBufs.begin(), readBufs.end());
    check(hrs_decode3(h_, in.data(), writeBufs.data(), erased.data(), static_cast<int>(erased.size()), len), h_);
  }

 protected:
  hrs_codec* h_ = nullptr;
};

// Host batches over a device set (hrs_encode_batch_host_multi /
// hrs_decode_batch_host_multi): one codec per device, equal contiguous stripe
// ranges, one host thread each. Layout and semantics as the single-codec
// calls (include/hrs.h).
inline void encodeBatchHostMulti(const std::vector<HipCode*>& codes, uint8_t* stripes, size_t rowStride,
                                 size_t stripeStride, size_t len, size_t nstripes) {
  std::vector<hrs_codec*> h;
  for (HipCode* c : codes) h.push_back(c->handle());
  check(hrs_encode_batch_host_multi(h.data(), static_cast<int>(h.size()), stripes, rowStride, stripeStride, len,
                                    nstripes),
        h.empty() ? nullptr : h[0]);
}

inline void decodeBatchHostMulti(const std::vector<HipCode*>& codes, const uint8_t* stripes, size_t rowStride,
                                 size_t stripeStride, const int* erased, int maxErased, uint8_t* out,
                                 size_t outRowStride, size_t outStripeStride, size_t len, size_t nstripes) {
  std::vector<hrs_codec*> h;
  for (HipCode* c : codes) h.push_back(c->handle());
  check(hrs_decode_batch_host_multi(h.data(), static_cast<int>(h.size()), stripes, rowStride, stripeStride, erased,
                                    maxErased, out, outRowStride, outStripeStride, len, nstripes),
        h.empty() ? nullptr : h[0]);
}

class HipReedSolomonCode : public HipCode {
 public:
  HipReedSolomonCode(int stripeSize, int paritySize, int device = -1)
      : HipCode(HRS_CODE_RS, stripeSize, paritySize, device) {}
};

class HipXORCode : public HipCode {
 public:
  explicit HipXORCode(int stripeSize, int device = -1) : HipCode(HRS_CODE_XOR, stripeSize, 1, device) {}
};

// NativeReedSolomonCode (the `nrs` codec, ISA-L Cauchy RS); decode outputs in
// the Java's order (hrs.h, HRS_CODE_NRS). symbolSize and decodeBulk3 throw,
// as UnsupportedOperationException / no such method in the Java.
// SimpleRegeneratingCode (the `src` codec): RS(k, r) + stored local XOR
// parities; srcParities = the codec's "parity_length_src".
class HipSimpleRegeneratingCode : public HipCode {
 public:
  HipSimpleRegeneratingCode(int stripeSize, int paritySize, int srcParities, int device = -1)
      : HipCode(HRS_CODE_SRC, stripeSize, paritySize, device, srcParities) {}
};

class HipNativeReedSolomonCode : public HipCode {
 public:
  HipNativeReedSolomonCode(int stripeSize, int paritySize, int device = -1)
      : HipCode(HRS_CODE_NRS, stripeSize, paritySize, device) {}
  int symbolSize() const override { throw std::logic_error("Not supported yet."); }
};

}  // namespace hrs
