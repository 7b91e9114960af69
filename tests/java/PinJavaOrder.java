// PinJavaOrder.java -- pins the Collect_Replicas order restatement against a
// real JVM (TEST INFRASTRUCTURE; not compiled in this image: no JDK).
//
// Replays tests/golden/java_order_cases.txt on the reference's own types --
// a java.util.HashMap keyed by org.javatuples.Pair<Integer,String>, as
// PeerData.Other_Replica_Gradients (PeerData.java:140) -- and prints, in the
// format of tests/golden/java_order_expected.txt, the Pair hashCode of every
// key put and the order of new ArrayList<>(keySet()) (IPLS.java:1218).
//
//   javac -cp javatuples-1.2.jar -d out tests/java/PinJavaOrder.java
//   java -cp out:javatuples-1.2.jar PinJavaOrder tests/golden/java_order_cases.txt > got.txt
//   diff got.txt tests/golden/java_order_expected.txt     # empty = the restatement is pinned
//
// The puts only insert absent keys, as Download_Scheduler.java:254-266 does
// (a stored key's array is folded into, the key is not put again).
import java.nio.charset.StandardCharsets;
import java.nio.file.Files;
import java.nio.file.Paths;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.List;
import java.util.Map;

import org.javatuples.Pair;

public final class PinJavaOrder {
    public static void main(String[] args) throws Exception {
        List<String> lines = Files.readAllLines(Paths.get(args[0]), StandardCharsets.UTF_8);
        Map<Pair<Integer, String>, double[]> m = new HashMap<>();
        StringBuilder out = new StringBuilder();
        for (String ln : lines) {
            if (ln.isEmpty()) continue;
            String[] f = ln.split(" ");
            switch (f[0]) {
                case "case":
                    out.append(ln).append('\n');
                    break;
                case "put": {
                    Pair<Integer, String> k = new Pair<>(Integer.parseInt(f[1]), f[2]);
                    if (!m.containsKey(k)) {
                        m.put(k, new double[0]);
                        out.append("hash ").append(f[1]).append(' ').append(f[2]).append(' ')
                           .append(k.hashCode()).append('\n');
                    }
                    break;
                }
                case "remove":
                    m.remove(new Pair<>(Integer.parseInt(f[1]), f[2]));
                    break;
                case "order": {
                    out.append("order");
                    for (Pair<Integer, String> k : new ArrayList<>(m.keySet()))
                        out.append(' ').append(k.getValue0()).append(':').append(k.getValue1());
                    out.append('\n');
                    break;
                }
                case "clear":
                    m = new HashMap<>();
                    break;
                default:
                    throw new IllegalArgumentException(ln);
            }
        }
        System.out.write(out.toString().getBytes(StandardCharsets.UTF_8));
        System.out.flush();
    }
}
