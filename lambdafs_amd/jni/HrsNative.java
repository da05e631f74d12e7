/*
 * JNI entry points of libhrs_jni.so (hrs_jni.c), shared by the engine's codec
 * classes. Mirrors the C ABI in include/hrs.h; the handle is an hrs_codec*.
 * Not compiled in this repository's CI (no JDK): see INTEGRATION.md.
 */
package io.hops.erasure_coding;

import java.io.IOException;

final class HrsNative {
  static final int CODE_RS = 0;   // HRS_CODE_RS
  static final int CODE_XOR = 1;  // HRS_CODE_XOR
  static final int CODE_NRS = 2;  // HRS_CODE_NRS
  static final int CODE_SRC = 3;  // HRS_CODE_SRC

  static {
    System.loadLibrary("hrs_jni");  // libhrs_jni.so -> libhrs.so
  }

  private HrsNative() {
  }

  // hrs_create_code / hrs_create_src on HIP device `device` (-1 = the
  // thread's current device; HipDevices.pick chooses it). A device that is
  // not visible throws IOException (HRS_EDEVICE), bad geometry
  // IllegalArgumentException.
  static native long create(int code, int stripeSize, int paritySize, int device) throws IOException;

  static native long createSrc(int stripeSize, int paritySize, int srcParitySize, int device) throws IOException;

  // hrs_device_count: HIP devices visible to this JVM (HIP_VISIBLE_DEVICES applies)
  static native int deviceCount();

  // hrs_codec_device: the device a handle runs on
  static native int device(long codec);

  static native void destroy(long codec);

  // hrs_locations_to_read_list; throws TooManyErasedLocations
  static native int[] locationsToRead(long codec, int[] erased) throws TooManyErasedLocations;

  static native void encode(long codec, byte[][] inputs, byte[][] outputs, int len) throws IOException;

  static native void decode(long codec, byte[][] readBufs, byte[][] writeBufs, int[] erased, int[] toRead,
      int[] notToRead, int len) throws IOException;

  static native void decode3(long codec, byte[][] readBufs, byte[][] writeBufs, int[] erased, int len)
      throws IOException;

  // hrs_encode_crc: crcs[k + p] (sources, then parities) continued in place
  static native void encodeCrc(long codec, byte[][] inputs, byte[][] outputs, int len, int[] crcs)
      throws IOException;

  // hrs_decode_crc: crcs[erased.length] continued in place over writeBufs
  static native void decodeCrc(long codec, byte[][] readBufs, byte[][] writeBufs, int[] erased, int[] toRead,
      int[] notToRead, int len, int[] crcs) throws IOException;

  // asynchronous rounds: hrs_encode_submit / hrs_decode_submit return a ticket
  // once the rows are staged; collect waits and copies the outputs (and, for
  // a checksummed round, continues crcs in place)
  static native long encodeSubmit(long codec, byte[][] inputs, int len, boolean checksums) throws IOException;

  static native long decodeSubmit(long codec, byte[][] readBufs, int[] erased, int[] toRead, int[] notToRead,
      int len, boolean checksums) throws IOException;

  static native void collect(long codec, long ticket, byte[][] outputs, int[] crcs) throws IOException;

  static native int pending(long codec);
}
