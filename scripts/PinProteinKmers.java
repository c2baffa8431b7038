// PinProteinKmers.java — pins, in one run, the three external semantics this build assumes
// (DESIGN.md §7). They live in un-vendored org.theseed artifacts (pom.xml:48-72), and no JDK
// or jar exists where this build was made, so this file is NOT compiled here. A maintainer
// with the jars runs scripts/pin_external_semantics.sh (a Java 11+ single-file launch):
//   java -cp "$SEED_JARS/*" scripts/PinProteinKmers.java tests/golden/pin > pin.txt
//   diff pin.txt tests/golden/pin/expected.txt
// An empty diff pins all three; a differing line names the assumption to change:
//   KMERS  new ProteinKmers(s) at the K apply uses (8: ApplyKmerProcessor.java:123 never calls
//          setKmerSize): the count iterated and the sorted distinct kmers. Assumed: the SET of
//          windows i = 0 .. L-8 inclusive, no filtering. An exclusive end shows as a missing
//          last kmer (then pass KMA_F_END_EXCLUSIVE, the JNI stub's `flags`); repeated windows
//          counted twice as count > distinct kmers (KMA_F_MULTISET).
//   FASTA  FastaInputStream records (BuildKmerProcessor.java:196-198): label, comment, sequence
//          of an edge-case file (CRLF / lone CR, blank lines, tab and double-space headers,
//          an empty record, an empty header, no final newline). Assumed: host/fasta.h's rules.
//   PEGS   Genome.getPegs() of a GTO whose pegs are out of id order with RNAs between them
//          (VERIFY row order, ApplyKmerProcessor.java:122). Assumed: the features array order.
import java.io.File;
import java.io.IOException;
import java.nio.file.Files;
import java.util.ArrayList;
import java.util.List;
import java.util.TreeSet;

import org.theseed.genome.Feature;
import org.theseed.genome.Genome;
import org.theseed.sequence.FastaInputStream;
import org.theseed.sequence.ProteinKmers;
import org.theseed.sequence.Sequence;

public class PinProteinKmers {
    public static void main(String[] args) throws IOException {
        File dir = new File(args.length > 0 ? args[0] : "tests/golden/pin");
        for (String prot : Files.readAllLines(new File(dir, "proteins.txt").toPath())) {
            ProteinKmers kmers = new ProteinKmers(prot);
            TreeSet<String> distinct = new TreeSet<>();
            int iterated = 0;
            for (String kmer : kmers) {
                distinct.add(kmer);
                iterated++;
            }
            System.out.println("KMERS\t" + prot + "\t" + iterated + "\t" + String.join(",", distinct));
        }
        try (FastaInputStream in = new FastaInputStream(new File(dir, "edge.faa"))) {
            for (Sequence seq : in)
                System.out.println("FASTA\t" + seq.getLabel() + "\t" + seq.getComment() + "\t"
                        + seq.getSequence());
        }
        Genome genome = new Genome(new File(dir, "shuffled.gto"));
        List<String> ids = new ArrayList<>();
        for (Feature peg : genome.getPegs())
            ids.add(peg.getId());
        System.out.println("PEGS\t" + genome.getId() + "\t" + String.join(",", ids));
    }
}
