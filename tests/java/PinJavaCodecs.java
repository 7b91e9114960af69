// PinJavaCodecs.java -- pins the restated Java-library behaviours of the
// aggregation path against a real JVM (TEST INFRASTRUCTURE; not compiled in
// this image: no JDK).
//
// Replays tests/golden/java_pin_cases.txt and prints, in the format of
// tests/golden/java_pin_expected.txt, what the JDK does: double addition and
// division as the reference's loops write them, ByteBuffer.putDouble,
// DataOutputStream.writeDouble, java.util.Base64's URL encoder/decoder,
// Marshall_Packet's frame bytes and ObjectOutputStream's bytes of a
// javatuples Pair<Integer,double[]>.
//
//   javac -cp javatuples-1.2.jar -d out tests/java/PinJavaCodecs.java
//   java -cp out:javatuples-1.2.jar PinJavaCodecs tests/golden/java_pin_cases.txt > got.txt
//   diff got.txt tests/golden/java_pin_expected.txt     # empty = pinned
import java.io.ByteArrayOutputStream;
import java.io.DataOutputStream;
import java.io.ObjectOutputStream;
import java.nio.ByteBuffer;
import java.nio.charset.StandardCharsets;
import java.nio.file.Files;
import java.nio.file.Paths;
import java.util.Base64;
import java.util.List;

import org.javatuples.Pair;

public final class PinJavaCodecs {
    static double[] doubles(String s) {
        if (s.equals("-")) return new double[0];
        String[] t = s.split(",");
        double[] d = new double[t.length];
        for (int i = 0; i < t.length; i++) d[i] = Double.longBitsToDouble(Long.parseUnsignedLong(t[i], 16));
        return d;
    }

    static String show(double[] d) {
        if (d.length == 0) return "-";
        StringBuilder b = new StringBuilder();
        for (int i = 0; i < d.length; i++) {
            if (i > 0) b.append(',');
            b.append(Double.isNaN(d[i]) ? "NaN" : String.format("%016x", Double.doubleToRawLongBits(d[i])));
        }
        return b.toString();
    }

    static String hex(byte[] b) {
        if (b.length == 0) return "-";
        StringBuilder s = new StringBuilder();
        for (byte x : b) s.append(String.format("%02x", x & 0xff));
        return s.toString();
    }

    static byte[] unhex(String s) {
        if (s.equals("-")) return new byte[0];
        byte[] b = new byte[s.length() / 2];
        for (int i = 0; i < b.length; i++) b[i] = (byte) Integer.parseInt(s.substring(2 * i, 2 * i + 2), 16);
        return b;
    }

    // Marshall_Packet(double[], OriginPeer, Partition, iteration, pid), MyIPFSClass.java:990-1016,
    // without the final Base64 (the b64enc cases pin that)
    static byte[] frame(double[] r, String origin, int partition, int iteration, short pid) {
        ByteBuffer buff = ByteBuffer.allocate(Double.BYTES * r.length + 3 * Integer.BYTES + Short.BYTES);
        buff.putShort(0, pid);
        buff.putInt(Short.BYTES, r.length);
        buff.putInt(Short.BYTES + Integer.BYTES, partition);
        buff.putInt(Short.BYTES + 2 * Integer.BYTES, iteration);
        for (int i = 0; i < r.length; i++) buff.putDouble(i * Double.BYTES + 3 * Integer.BYTES + Short.BYTES, r[i]);
        byte[] barr = new byte[buff.remaining()];
        byte[] id = origin.getBytes();
        buff.get(barr);
        byte[] fin = new byte[barr.length + origin.length()];
        for (int i = 0; i < barr.length; i++) fin[i] = barr[i];
        for (int i = barr.length; i < fin.length; i++) fin[i] = id[i - barr.length];
        return fin;
    }

    public static void main(String[] args) throws Exception {
        List<String> lines = Files.readAllLines(Paths.get(args[0]), StandardCharsets.UTF_8);
        StringBuilder out = new StringBuilder();
        for (String ln : lines) {
            if (ln.isEmpty()) continue;
            String[] f = ln.split(" ");
            String ans;
            switch (f[0]) {
                case "fold": {                                   // Updater.java:115-117
                    double[] acc = doubles(f[1]), g = doubles(f[2]);
                    for (int i = 0; i < acc.length; i++) acc[i] = acc[i] + g[i];
                    ans = show(acc);
                    break;
                }
                case "divide": {                                 // IPLS.java:1162-1171
                    double[] w = doubles(f[1]);
                    boolean secure = f[2].equals("1");
                    double[] o = new double[w.length - 1];
                    for (int j = 0; j < w.length - 1; j++) {
                        if (w[w.length - 1] == 0.0) o[j] = w[j];
                        else if (secure) o[j] = w[j] / (Math.pow(10, 12) * w[w.length - 1]);
                        else o[j] = w[j] / w[w.length - 1];
                    }
                    ans = show(o);
                    break;
                }
                case "putdouble": {
                    ByteBuffer b = ByteBuffer.allocate(8);
                    b.putDouble(Double.longBitsToDouble(Long.parseUnsignedLong(f[1], 16)));
                    ans = hex(b.array());
                    break;
                }
                case "writedouble": {
                    ByteArrayOutputStream bo = new ByteArrayOutputStream();
                    DataOutputStream d = new DataOutputStream(bo);
                    d.writeDouble(Double.longBitsToDouble(Long.parseUnsignedLong(f[1], 16)));
                    d.flush();
                    ans = hex(bo.toByteArray());
                    break;
                }
                case "b64enc": {
                    String t = Base64.getUrlEncoder().encodeToString(unhex(f[1]));
                    ans = t.isEmpty() ? "-" : t;
                    break;
                }
                case "b64dec":
                    try {
                        ans = hex(Base64.getUrlDecoder().decode(f[1].getBytes(StandardCharsets.US_ASCII)));
                    } catch (IllegalArgumentException e) {
                        ans = "IAE";
                    }
                    break;
                case "frame":
                    ans = hex(frame(doubles(f[5]), f[4], Integer.parseInt(f[2]), Integer.parseInt(f[3]),
                                    Short.parseShort(f[1])));
                    break;
                case "pair": {                                   // MyIPFSClass.java:160-166
                    ByteArrayOutputStream bo = new ByteArrayOutputStream();
                    ObjectOutputStream oos = new ObjectOutputStream(bo);
                    oos.writeObject(new Pair<Integer, double[]>(Integer.parseInt(f[1]), doubles(f[2])));
                    oos.close();
                    ans = hex(bo.toByteArray());
                    break;
                }
                default:
                    throw new IllegalArgumentException(ln);
            }
            out.append(f[0]).append(' ').append(ans).append('\n');
        }
        System.out.write(out.toString().getBytes(StandardCharsets.UTF_8));
        System.out.flush();
    }
}
