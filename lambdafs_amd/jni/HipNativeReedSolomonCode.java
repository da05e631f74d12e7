/*
 * Drop-in for io.hops.erasure_coding.NativeReedSolomonCode (the `nrs` codec,
 * hops-erasure-coding/.../NativeReedSolomonCode.java:32-196) on MI355X: select with
 *   hdfs.raid.erasure.code.nrs = io.hops.erasure_coding.HipNativeReedSolomonCode.
 * Same Cauchy RS code as libhadoop's ISA-L coder (erasure_coder.c) and the same
 * decode output ordering (writeBufs[i] = i-th not-to-read location in Apache
 * [data, parity] order); no direct-buffer copies, bulk math in libhrs.so (HRS_CODE_NRS).
 */
package io.hops.erasure_coding;

import java.io.IOException;
import org.apache.hadoop.conf.Configurable;
import org.apache.hadoop.conf.Configuration;

public class HipNativeReedSolomonCode extends ErasureCode implements Configurable {
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

  private static long create(int code, int k, int p, int device) {
    try {
      return HrsNative.create(code, k, p, device);
    } catch (IOException e) {  // no such device: init(Codec) declares no IOException
      throw new RuntimeException(e);
    }
  }

  public HipNativeReedSolomonCode() {
  }

  @Override
  public void init(Codec codec) {  // NativeReedSolomonCode.java:44-51, :175-181
    release();
    stripeSize = codec.stripeLength;
    paritySize = codec.parityLength;
    nativeCodec = create(HrsNative.CODE_NRS, stripeSize, paritySize, HipDevices.pick(conf));
  }

  @Override
  public void encodeBulk(byte[][] inputs, byte[][] outputs) throws IOException {  // :55-88
    HrsNative.encode(nativeCodec, inputs, outputs, inputs[0].length);
  }

  @Override
  public void decodeBulk(byte[][] readBufs, byte[][] writeBufs, int[] erasedLocations,
      int[] locationsToRead, int[] locationsNotToRead) throws IOException {  // :90-152
    HrsNative.decode(nativeCodec, readBufs, writeBufs, erasedLocations, locationsToRead,
        locationsNotToRead, readBufs[0].length);
  }

  @Override
  public void encode(int[] message, int[] parity) {
    throw new UnsupportedOperationException("Not supported yet.");
  }

  @Override
  public void decode(int[] data, int[] erasedLocations, int[] erasedValues) {
    throw new UnsupportedOperationException("Not supported yet.");
  }

  @Override
  public void decode(int[] data, int[] erasedLocations, int[] erasedValues, int[] locationsToRead,
      int[] locationsNotToRead) {
    throw new UnsupportedOperationException("Not supported yet.");
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
    throw new UnsupportedOperationException("Not supported yet.");
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
