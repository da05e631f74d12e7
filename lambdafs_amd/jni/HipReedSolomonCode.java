/*
 * The Java side of the drop-in: a codec class for the hops erasure-coding
 * plugin surface (hadoop-hdfs/src/main/java/io/hops/erasure_coding/
 * ErasureCode.java:25-182), to be added to
 * hops-erasure-coding-project/hops-erasure-coding/src/main/java/io/hops/erasure_coding/
 * and selected with  hdfs.raid.erasure.code.rs = io.hops.erasure_coding.HipReedSolomonCode
 * (Codec.java:52-53, :200-213). Semantics are those of ReedSolomonCode, bit-exact;
 * every byte is computed by libhrs.so (MI355X) through libhrs_jni.so.
 *
 * Not compiled in this repository's CI (no JDK in the build image): see
 * INTEGRATION.md for the build recipe.
 */
package io.hops.erasure_coding;

import java.io.IOException;
import java.io.UncheckedIOException;
import java.util.Arrays;
import org.apache.hadoop.conf.Configurable;
import org.apache.hadoop.conf.Configuration;

/*
 * Extends ReedSolomonCode itself, so it is a drop-in wherever the reference
 * code or its tests expect that class: `instanceof ReedSolomonCode`
 * (TestCodec.java:119), the cast to reach the 3-arg decodeBulk
 * (TestNativeErasureCodes.java:100), and the inherited Java
 * computeErrorLocations (ReedSolomonCode.java:243-287; its inner decode call
 * runs on the GPU through the override below). super.init sets up the
 * reference's own small tables for that method; every bulk byte is still
 * computed by libhrs.so. ReedSolomonCode's bulk methods declare no checked
 * exceptions, so an engine failure surfaces as UncheckedIOException (its
 * cause the IOException the shim threw), as the scalar methods already did.
 */
public class HipReedSolomonCode extends ReedSolomonCode implements Configurable {
  private long nativeCodec;  // hrs_codec*, owned (cf. jni_common.c:35-70 "nativeCoder")
  private int stripeSize;
  private int paritySize;

  // Configurable: Codec.createErasureCode hands the conf over before init
  // (ReflectionUtils.newInstance, Codec.java:209-211); init then takes the
  // next device of hdfs.raid.hip.devices (HipDevices).
  private Configuration conf;

  @Override
  public void setConf(Configuration conf) {
    this.conf = conf;
  }

  @Override
  public Configuration getConf() {
    return conf;
  }

  /** The HIP device this instance runs on. */
  public int device() {
    return HrsNative.device(nativeCodec);
  }

  private static long create(int code, int k, int p, int device) {
    try {
      return HrsNative.create(code, k, p, device);
    } catch (IOException e) {  // no such device: init(Codec) declares no IOException
      throw new RuntimeException(e);
    }
  }

  public HipReedSolomonCode() {
  }

  @Deprecated
  public HipReedSolomonCode(int stripeSize, int paritySize) {
    super(stripeSize, paritySize);  // the reference's tables (computeErrorLocations)
    init(stripeSize, paritySize);
  }

  @Override
  public void init(Codec codec) {  // ReedSolomonCode.java:48-54
    super.init(codec);  // the reference's tables (computeErrorLocations)
    init(codec.stripeLength, codec.parityLength);
  }

  private synchronized void init(int stripeSize, int paritySize) {
    release();
    this.stripeSize = stripeSize;
    this.paritySize = paritySize;
    this.nativeCodec = create(HrsNative.CODE_RS, stripeSize, paritySize, HipDevices.pick(conf));
  }

  /** Same result as ReedSolomonCode.encodeBulk (ReedSolomonCode.java:103-125). */
  @Override
  public void encodeBulk(byte[][] inputs, byte[][] outputs) {
    assert (stripeSize == inputs.length);
    assert (paritySize == outputs.length);
    try {
      HrsNative.encode(nativeCodec, inputs, outputs, outputs[0].length);
    } catch (IOException e) {
      throw new UncheckedIOException(e);
    }
    // The Java bulk remainder zeroes its inputs (GaloisField.java:326-338); keep that contract.
    for (byte[] in : inputs) {
      Arrays.fill(in, (byte) 0);
    }
  }

  /**
   * encodeBulk plus the block checksums Encoder.encodeStripe keeps with
   * computeBlockChecksum (Encoder.java:408-450): crcs[k + p] holds the running
   * CRC32 values (sources, then parities; getValue() truncated to int, 0 for a
   * fresh CRC32) and is updated in place, so the Encoder's updateChecksums and
   * parityChecksums passes over the heap buffers go away.
   */
  public void encodeBulkWithChecksums(byte[][] inputs, byte[][] outputs, int[] crcs) throws IOException {
    assert (stripeSize == inputs.length);
    assert (paritySize == outputs.length);
    HrsNative.encodeCrc(nativeCodec, inputs, outputs, outputs[0].length, crcs);
    for (byte[] in : inputs) {
      Arrays.fill(in, (byte) 0);
    }
  }

  /**
   * 5-arg decodeBulk plus the CRC32 of each repaired buffer, continued in
   * crcs[erasedLocations.length] (Decoder.java:222-229, :645-655).
   */
  public void decodeBulkWithChecksums(byte[][] readBufs, byte[][] writeBufs, int[] erasedLocations,
      int[] locationsToRead, int[] locationsNotToRead, int[] crcs) throws IOException {
    if (erasedLocations.length == 0) {
      return;
    }
    HrsNative.decodeCrc(nativeCodec, readBufs, writeBufs, erasedLocations, locationsToRead,
        locationsNotToRead, readBufs[0].length, crcs);
  }

  /**
   * Asynchronous rounds for a caller that keeps the GPU busy across rounds
   * (Encoder.java:421-453 runs encodeBulk rounds back to back): the round is
   * staged and queued, and the caller may reuse `inputs` at once (they are
   * zeroed, as encodeBulk does); collect(ticket, writeBufs) later waits for it.
   * Up to 4 rounds may be outstanding per codec.
   */
  public long encodeBulkAsync(byte[][] inputs) throws IOException {
    long t = HrsNative.encodeSubmit(nativeCodec, inputs, inputs[0].length, false);
    for (byte[] in : inputs) {
      Arrays.fill(in, (byte) 0);
    }
    return t;
  }

  /** encodeBulkAsync plus the block checksums, continued by collect(ticket, outputs, crcs). */
  public long encodeBulkAsyncWithChecksums(byte[][] inputs) throws IOException {
    long t = HrsNative.encodeSubmit(nativeCodec, inputs, inputs[0].length, true);
    for (byte[] in : inputs) {
      Arrays.fill(in, (byte) 0);
    }
    return t;
  }

  /** The 5-arg decodeBulk round, submitted (Decoder.java:352-353). */
  public long decodeBulkAsync(byte[][] readBufs, int[] erasedLocations, int[] locationsToRead,
      int[] locationsNotToRead, boolean checksums) throws IOException {
    return HrsNative.decodeSubmit(nativeCodec, readBufs, erasedLocations, locationsToRead, locationsNotToRead,
        readBufs[0].length, checksums);
  }

  /** Waits for a submitted round and copies its output rows into `outputs`. */
  public void collect(long ticket, byte[][] outputs) throws IOException {
    HrsNative.collect(nativeCodec, ticket, outputs, null);
  }

  /** collect for a checksummed round: crcs (k + p or one per erased location) continued in place. */
  public void collect(long ticket, byte[][] outputs, int[] crcs) throws IOException {
    HrsNative.collect(nativeCodec, ticket, outputs, crcs);
  }

  /** Same result as ReedSolomonCode.decodeBulk 5-arg (ReedSolomonCode.java:191-211). */
  @Override
  public void decodeBulk(byte[][] readBufs, byte[][] writeBufs, int[] erasedLocations,
      int[] locationsToRead, int[] locationsNotToRead) {
    if (erasedLocations.length == 0) {
      return;
    }
    try {
      HrsNative.decode(nativeCodec, readBufs, writeBufs, erasedLocations, locationsToRead,
          locationsNotToRead, readBufs[0].length);
    } catch (IOException e) {
      throw new UncheckedIOException(e);
    }
  }

  /** Same result as ReedSolomonCode.decodeBulk 3-arg (ReedSolomonCode.java:168-185). */
  @Override
  public void decodeBulk(byte[][] readBufs, byte[][] writeBufs, int[] erasedLocation) {
    if (erasedLocation.length == 0) {
      return;
    }
    try {
      HrsNative.decode3(nativeCodec, readBufs, writeBufs, erasedLocation, readBufs[0].length);
    } catch (IOException e) {
      throw new UncheckedIOException(e);
    }
  }

  @Override
  public void encode(int[] message, int[] parity) {  // ReedSolomonCode.java:84-97
    byte[][] in = new byte[stripeSize][1];
    byte[][] out = new byte[paritySize][1];
    for (int i = 0; i < stripeSize; i++) {
      in[i][0] = (byte) message[i];
    }
    try {
      HrsNative.encode(nativeCodec, in, out, 1);
    } catch (IOException e) {
      throw new RuntimeException(e);
    }
    for (int i = 0; i < paritySize; i++) {
      parity[i] = out[i][0] & 0xFF;
    }
  }

  @Override
  public void decode(int[] data, int[] erasedLocations, int[] erasedValues) {  // :127-142
    if (erasedLocations.length == 0) {
      return;
    }
    // zero data at the erased locations, then the 3-arg bulk decode of the
    // zeroed column: erasedValues[i] = solution i of the Vandermonde solve
    // (with a repeated location the 5-arg form's matching would copy the
    // first one's value instead)
    for (int loc : erasedLocations) {
      data[loc] = 0;
    }
    byte[][] rows = new byte[data.length][1];
    for (int i = 0; i < data.length; i++) {
      rows[i][0] = (byte) data[i];
    }
    byte[][] out = new byte[erasedLocations.length][1];
    try {
      HrsNative.decode3(nativeCodec, rows, out, erasedLocations, 1);
    } catch (IOException e) {
      throw new RuntimeException(e);
    }
    for (int i = 0; i < erasedLocations.length; i++) {
      erasedValues[i] = out[i][0] & 0xFF;
    }
  }

  @Override
  public void decode(int[] data, int[] erasedLocations, int[] erasedValues,
      int[] locationsToRead, int[] locationsNotToRead) {  // :144-166
    for (int loc : locationsNotToRead) {
      data[loc] = 0;  // the Java zeroes data at the decoded locations
    }
    byte[][] rows = new byte[data.length][1];
    for (int i = 0; i < data.length; i++) {
      rows[i][0] = (byte) data[i];
    }
    byte[][] out = new byte[erasedLocations.length][1];
    try {
      HrsNative.decode(nativeCodec, rows, out, erasedLocations, locationsToRead, locationsNotToRead, 1);
    } catch (IOException e) {
      throw new RuntimeException(e);
    }
    // ReedSolomonCode.java:158-165 copies a recovered value only where
    // erasedLocations[i] is one of locationsNotToRead; any other entry of
    // erasedValues keeps what the caller passed (the engine's zero row for it
    // is not copied).
    for (int i = 0; i < erasedLocations.length; i++) {
      for (int loc : locationsNotToRead) {
        if (erasedLocations[i] == loc) {
          erasedValues[i] = out[i][0] & 0xFF;
          break;
        }
      }
    }
  }

  @Override
  public int stripeSize() {
    return stripeSize;
  }

  @Override
  public int paritySize() {
    return paritySize;
  }

  @Override
  public int symbolSize() {
    return 8;
  }

  public synchronized void release() {
    if (nativeCodec != 0) {
      HrsNative.destroy(nativeCodec);
      nativeCodec = 0;
    }
  }

  @Override
  protected void finalize() throws Throwable {
    release();
    super.finalize();
  }
}
