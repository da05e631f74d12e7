/*
 * Drop-in for io.hops.erasure_coding.XORCode (hops-erasure-coding/.../XORCode.java:24-146)
 * on MI355X: select with  hdfs.raid.erasure.code.xor = io.hops.erasure_coding.HipXORCode.
 * Bulk paths run in libhrs.so (HRS_CODE_XOR); results are bit-identical to XORCode.
 */
package io.hops.erasure_coding;

import java.io.IOException;
import org.apache.hadoop.conf.Configurable;
import org.apache.hadoop.conf.Configuration;

public class HipXORCode extends ErasureCode implements Configurable {
  private long nativeCodec;
  private int stripeSize;

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

  public HipXORCode() {
  }

  @Override
  public void init(Codec codec) {  // XORCode.java:40-51
    assert (codec.parityLength == 1);
    release();
    stripeSize = codec.stripeLength;
    nativeCodec = create(HrsNative.CODE_XOR, codec.stripeLength, 1, HipDevices.pick(conf));
  }

  @Override
  public void encodeBulk(byte[][] inputs, byte[][] outputs) throws IOException {  // :99-113
    HrsNative.encode(nativeCodec, inputs, outputs, outputs[0].length);
  }

  @Override
  public void decodeBulk(byte[][] readBufs, byte[][] writeBufs, int[] erasedLocations,
      int[] locationsToRead, int[] locationsNotToRead) throws IOException {  // :140-145
    HrsNative.decode3(nativeCodec, readBufs, writeBufs, erasedLocations, readBufs[0].length);
  }

  @Override
  public void encode(int[] message, int[] parity) {  // :54-61 (scalar, no device round trip)
    parity[0] = message[0];
    for (int i = 1; i < message.length; i++) {
      parity[0] ^= message[i];
    }
  }

  @Override
  public void decode(int[] data, int[] erasedLocation, int[] erasedValue) {  // :63-77
    if (erasedLocation.length != 1) {
      return;
    }
    int val = 0;
    for (int i = 0; i < data.length; i++) {
      if (i != erasedLocation[0]) {
        val ^= data[i];
      }
    }
    erasedValue[0] = val;
  }

  @Override
  public void decode(int[] data, int[] erasedLocations, int[] erasedValues, int[] locationsToRead,
      int[] locationsNotToRead) {
    decode(data, erasedLocations, erasedValues);
  }

  @Override
  public int stripeSize() {
    return stripeSize;
  }

  @Override
  public int paritySize() {
    return 1;
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
