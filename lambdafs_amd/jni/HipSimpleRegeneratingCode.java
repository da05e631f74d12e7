/*
 * Drop-in for io.hops.erasure_coding.SimpleRegeneratingCode (the `src` codec,
 * hops-erasure-coding/.../SimpleRegeneratingCode.java:28-482) on MI355X: select with
 *   hdfs.raid.erasure.code.src = io.hops.erasure_coding.HipSimpleRegeneratingCode.
 * Bulk calls (ErasureCode's per-column loops over the Java's encode/decode) run as
 * GF(2^8) matrices in libhrs.so (HRS_CODE_SRC); locationsToReadForDecode is the
 * product's restatement (hrs_locations_to_read_list). Bit-identical parity and repairs.
 */
package io.hops.erasure_coding;

import java.io.IOException;
import java.util.ArrayList;
import java.util.List;
import org.json.JSONException;
import org.apache.hadoop.conf.Configurable;
import org.apache.hadoop.conf.Configuration;

public class HipSimpleRegeneratingCode extends ErasureCode implements Configurable {
  private long nativeCodec;
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

  private static long createSrc(int k, int p, int s, int device) {
    try {
      return HrsNative.createSrc(k, p, s, device);
    } catch (IOException e) {  // no such device: init(Codec) declares no IOException
      throw new RuntimeException(e);
    }
  }

  public HipSimpleRegeneratingCode() {
  }

  @Override
  public void init(Codec codec) {  // SimpleRegeneratingCode.java:52-64
    int srcParities = 0;
    try {
      srcParities = codec.json.getInt("parity_length_src");
    } catch (JSONException e) {
      srcParities = 0;  // the Java logs and keeps 0
    }
    release();
    stripeSize = codec.stripeLength;
    paritySize = codec.parityLength;
    nativeCodec = createSrc(stripeSize, paritySize, srcParities, HipDevices.pick(conf));
  }

  @Override
  public void encodeBulk(byte[][] inputs, byte[][] outputs) throws IOException {  // ErasureCode.java:136-156
    HrsNative.encode(nativeCodec, inputs, outputs, outputs[0].length);
  }

  @Override
  public void decodeBulk(byte[][] readBufs, byte[][] writeBufs, int[] erasedLocations,
      int[] locationsToRead, int[] locationsNotToRead) throws IOException {  // ErasureCode.java:162-181
    HrsNative.decode(nativeCodec, readBufs, writeBufs, erasedLocations, locationsToRead,
        locationsNotToRead, readBufs[0].length);
  }

  @Override
  public List<Integer> locationsToReadForDecode(List<Integer> erasedLocations)
      throws TooManyErasedLocations {  // SimpleRegeneratingCode.java:300-366
    int[] erased = new int[erasedLocations.size()];
    for (int i = 0; i < erased.length; i++) {
      erased[i] = erasedLocations.get(i);
    }
    int[] r = HrsNative.locationsToRead(nativeCodec, erased);
    List<Integer> out = new ArrayList<Integer>(r.length);
    for (int x : r) {
      out.add(x);
    }
    return out;
  }

  @Override
  public void encode(int[] message, int[] parity) {  // :116-157, one symbol column
    byte[][] in = new byte[message.length][1];
    byte[][] out = new byte[parity.length][1];
    for (int i = 0; i < message.length; i++) {
      in[i][0] = (byte) message[i];
    }
    try {
      HrsNative.encode(nativeCodec, in, out, 1);
    } catch (IOException e) {
      throw new RuntimeException(e);
    }
    for (int i = 0; i < parity.length; i++) {
      parity[i] = out[i][0] & 0xFF;
    }
  }

  @Override
  public void decode(int[] data, int[] erasedLocations, int[] erasedValues) {
    // :188-191 runs an RS decode over the whole stripe (indexing past its
    // tables for locations >= k + r); not provided.
    throw new UnsupportedOperationException("3-argument SimpleRegeneratingCode.decode");
  }

  @Override
  public void decode(int[] data, int[] erasedLocations, int[] erasedValues, int[] locationsToRead,
      int[] locationsNotToRead) {  // :194-277, one symbol column
    byte[][] in = new byte[data.length][1];
    byte[][] out = new byte[erasedLocations.length][1];
    for (int i = 0; i < data.length; i++) {
      in[i][0] = (byte) data[i];
    }
    try {
      HrsNative.decode(nativeCodec, in, out, erasedLocations, locationsToRead, locationsNotToRead, 1);
    } catch (IOException e) {
      throw new RuntimeException(e);
    }
    for (int i = 0; i < erasedValues.length; i++) {
      erasedValues[i] = out[i][0] & 0xFF;
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
