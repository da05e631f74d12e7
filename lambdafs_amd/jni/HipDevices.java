/*
 * Device set of the HIP codec classes: which GPU each codec instance of this
 * JVM runs on.
 *
 * The hops EC stack creates one codec per Encoder / Decoder (Encoder.java:80,
 * Decoder.java:90) through Codec.createErasureCode, which instantiates the
 * class with ReflectionUtils.newInstance(erasureCode, conf) -- calling
 * setConf(conf) on a Configurable codec -- and then init(this)
 * (hadoop-hdfs/src/main/java/io/hops/erasure_coding/Codec.java:200-213).
 * The HIP codecs are Configurable; at init each takes the next device of
 *
 *   hdfs.raid.hip.devices = <ordinals or ranges, e.g. "0,2,4-7">   (default: every visible device)
 *
 * round robin over the JVM, so the mapper threads of one task JVM spread
 * over the node's GPUs. A JVM confined with HIP_VISIBLE_DEVICES sees only its
 * devices, renumbered from 0 (INTEGRATION.md §3). Ordinals are checked by the
 * engine: a device that does not exist fails the codec's creation with an
 * IOException (wrapped in a RuntimeException by init, which may not throw it).
 * Same rules as the Python mirror (lambdafs_amd/devset.py).
 */
package io.hops.erasure_coding;

import java.util.ArrayList;
import java.util.List;
import java.util.concurrent.atomic.AtomicInteger;
import org.apache.hadoop.conf.Configuration;

final class HipDevices {
  static final String DEVICES_KEY = "hdfs.raid.hip.devices";

  private static final AtomicInteger NEXT = new AtomicInteger();

  private HipDevices() {
  }

  /** The ordinals a hdfs.raid.hip.devices value names, in order. */
  static int[] parse(String spec, int visible) {
    if (spec == null || spec.trim().isEmpty() || spec.trim().equalsIgnoreCase("all")) {
      if (visible <= 0) {
        throw new IllegalStateException("no HIP device visible for " + DEVICES_KEY);
      }
      int[] all = new int[visible];
      for (int i = 0; i < visible; i++) {
        all[i] = i;
      }
      return all;
    }
    List<Integer> out = new ArrayList<Integer>();
    for (String part : spec.split(",", -1)) {
      String t = part.trim();
      int dash = t.indexOf('-');
      try {
        int lo = Integer.parseInt(dash < 0 ? t : t.substring(0, dash).trim());
        int hi = dash < 0 ? lo : Integer.parseInt(t.substring(dash + 1).trim());
        if (lo < 0 || hi < lo) {
          throw new IllegalArgumentException(DEVICES_KEY + ": bad entry '" + t + "'");
        }
        for (int d = lo; d <= hi; d++) {
          out.add(d);
        }
      } catch (NumberFormatException e) {
        throw new IllegalArgumentException(DEVICES_KEY + ": bad entry '" + t + "'", e);
      }
    }
    int[] r = new int[out.size()];
    for (int i = 0; i < r.length; i++) {
      r[i] = out.get(i);
    }
    return r;
  }

  /** The device of the next codec instance: -1 (current device) without a conf. */
  static int pick(Configuration conf) {
    if (conf == null) {
      return -1;
    }
    String spec = conf.get(DEVICES_KEY);
    boolean all = spec == null || spec.trim().isEmpty() || spec.trim().equalsIgnoreCase("all");
    int[] set = parse(spec, all ? HrsNative.deviceCount() : 0);
    return set[Math.floorMod(NEXT.getAndIncrement(), set.length)];
  }
}
